"""Shape fuzzing of the implicit-GEMM convolution kernels (hypothesis, bounded examples):
random N/H/W/C/K/R/stride/pad (channels multiples of 8, tails on every tile edge), all
three passes vs fp32 torch."""
import pytest
import torch
import torch.nn.functional as F

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


@settings(max_examples=25, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(N=st.integers(1, 5), H=st.integers(3, 13), W=st.integers(3, 13), C8=st.integers(1, 12),
       K8=st.integers(1, 20), R=st.sampled_from([1, 3]), stride=st.sampled_from([1, 2]), cfg=st.integers(-1, 3))
def test_conv_fuzz(gpu, N, H, W, C8, K8, R, stride, cfg):
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    C, K = 8 * C8, 8 * K8
    pad = R // 2
    g = torch.Generator().manual_seed(N * 7919 + H * 131 + W * 17 + C + K + R + stride)
    x = torch.randn(N, C, H, W, generator=g).cuda().bfloat16()
    w = (torch.randn(K, C, R, R, generator=g) / (C * R * R) ** 0.5).cuda().bfloat16()
    xf = x.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    ref = F.conv2d(xf, wf, stride=stride, padding=pad)
    dy = torch.randn(ref.shape, generator=g).cuda().bfloat16()
    ref.backward(dy.float())
    xh, wh = x.permute(0, 2, 3, 1).contiguous(), w.permute(0, 2, 3, 1).contiguous()
    y, _ = m.conv_fwd(xh, wh, stride, pad, True, cfg)
    assert _rel(y.permute(0, 3, 1, 2), ref.detach()) < 1.5e-2
    dyh = dy.permute(0, 2, 3, 1).contiguous()
    dx = m.conv_dgrad(dyh, wh.permute(3, 1, 2, 0).contiguous(), H, W, stride, pad, cfg)
    assert _rel(dx.permute(0, 3, 1, 2), xf.grad) < 1.5e-2
    dw = m.conv_wgrad(dyh, xh, R, R, stride, pad, 0, cfg)
    assert _rel(dw.permute(0, 3, 1, 2), wf.grad) < 1.5e-2
