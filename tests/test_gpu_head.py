"""Native projection head (ops/head.py), fused row normalisation and norm statistics
(csrc/kernels/featnorm.hip) vs plain PyTorch fp32/autograd references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _m():
    from simclr_pytorch_distributed_amd.ops import _ext
    return _ext.require()


@pytest.mark.parametrize("D", [64, 128, 256, 100])
def test_row_normalize_matches_torch(gpu, D):
    from simclr_pytorch_distributed_amd.ops.contrastive import row_normalize
    torch.manual_seed(0)
    x = torch.randn(333, D, device=gpu)
    x[5] = 0.0                                    # clamped row (norm < eps)
    x[7] *= 1e-14
    xa = x.clone().requires_grad_(True)
    xb = x.double().clone().requires_grad_(True)
    ya = row_normalize(xa)
    yb = F.normalize(xb, dim=1)
    assert torch.allclose(ya.double(), yb, rtol=1e-6, atol=1e-6)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g.double())
    assert torch.allclose(xa.grad.double(), xb.grad, rtol=1e-4, atol=1e-4 * xb.grad.abs().max().item())


@pytest.mark.parametrize("shape", [(512, 128), (300, 100), (8192, 128)])
@pytest.mark.parametrize("momentum", [1.0, 0.9])
def test_norm_stats_matches_torch(gpu, momentum, shape):
    m = _m()
    torch.manual_seed(1)
    x = torch.randn(*shape, device=gpu) * 3
    rec = torch.zeros((), device=gpu)
    valid = torch.zeros((), device=gpu)
    sums = torch.zeros(2, dtype=torch.float64, device=gpu)
    ref_rec = None
    for step in range(3):
        xs = x * (1 + 0.1 * step)
        out = m.norm_stats(xs, 1, sums, float(xs.shape[0]), momentum, rec, valid)
        nrm = xs.double().norm(dim=1)
        mean = nrm.mean()
        var = (nrm * nrm).mean() - mean * mean
        ref_rec = mean if ref_rec is None else (1 - momentum) * ref_rec + momentum * mean
        sec = ((nrm - ref_rec) ** 2).sum() / nrm.numel()
        l2 = (nrm ** 2).sum() / nrm.numel()
        exp = torch.stack([mean, var, ref_rec, sec, l2]).float()
        assert torch.allclose(out, exp, rtol=1e-4, atol=1e-4), (out, exp)
        assert torch.allclose(rec, ref_rec.float(), rtol=1e-5)
        assert valid.item() == 1.0


def test_norm_stats_two_phase(gpu):
    """mode 0 (local sums) + mode 2 (finalize from given sums) == mode 1 for W=1."""
    m = _m()
    x = torch.randn(256, 128, device=gpu)
    r1, v1 = torch.zeros((), device=gpu), torch.zeros((), device=gpu)
    r2, v2 = torch.zeros((), device=gpu), torch.zeros((), device=gpu)
    s1 = torch.zeros(2, dtype=torch.float64, device=gpu)
    s2 = torch.zeros(2, dtype=torch.float64, device=gpu)
    a = m.norm_stats(x, 1, s1, 256.0, 1.0, r1, v1)
    m.norm_stats(x, 0, s2, 256.0, 1.0, r2, v2)
    b = m.norm_stats(x, 2, s2, 256.0, 1.0, r2, v2)
    assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("head", ["mlp", "linear"])
def test_native_head_matches_autograd(gpu, head):
    from simclr_pytorch_distributed_amd.models.executor import head_forward
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    from simclr_pytorch_distributed_amd.ops.head import projection_head
    from simclr_pytorch_distributed_amd.ops.weights import ConvWeightCache
    torch.manual_seed(2)
    a = SupConResNet("resnet50", head=head).to(gpu)
    b = SupConResNet("resnet50", head=head).to(gpu)
    b.load_state_dict(a.state_dict())
    lins = [mm for mm in a.head.modules() if isinstance(mm, torch.nn.Linear)]
    wc = ConvWeightCache(lins, None)
    wc.refresh()
    feat = torch.randn(64, 2048, device=gpu)
    fa = feat.clone().requires_grad_(True)
    fb = feat.clone().requires_grad_(True)
    za = projection_head(fa, a.head, wc)
    zb = head_forward(b.head, fb)
    assert za.dtype == torch.float32
    assert torch.allclose(za, zb, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(za)
    za.backward(g)
    zb.backward(g)
    rel = lambda u, v: ((u - v).norm() / v.norm().clamp_min(1e-12)).item()  # noqa: E731
    assert rel(fa.grad, fb.grad) < 1e-2
    for pa, pb in zip(a.head.parameters(), b.head.parameters()):
        assert pa.grad is not None
        assert rel(pa.grad, pb.grad) < 1e-2


@pytest.mark.parametrize("rows,din,dout,head", [(77, 512, 64, "mlp"), (256, 2048, 128, "mlp"), (40, 256, 128, "linear")])
def test_native_head_vs_fp32(gpu, rows, din, dout, head):
    """Hand-written head GEMMs (igemm 1x1 + fused bias/ReLU/fp32 epilogues, ReLU-backward
    store + bias column sums) vs a plain fp32 torch autograd reference of the same head."""
    import torch.nn as nn
    from simclr_pytorch_distributed_amd.ops.head import projection_head
    from simclr_pytorch_distributed_amd.ops.weights import ConvWeightCache
    torch.manual_seed(3)
    if head == "mlp":
        mod = nn.Sequential(nn.Linear(din, din), nn.ReLU(inplace=True), nn.Linear(din, dout)).to(gpu)
        with torch.no_grad():
            for lin in (mod[0], mod[2]):
                lin.bias.uniform_(-0.5, 0.5)   # biases large enough to matter
    else:
        mod = nn.Linear(din, dout).to(gpu)
    ref = __import__("copy").deepcopy(mod)
    lins = [m for m in mod.modules() if isinstance(m, nn.Linear)]
    wc = ConvWeightCache(lins, None)
    wc.refresh()
    feat = torch.randn(rows, din, device=gpu)
    fa = feat.clone().requires_grad_(True)
    fr = feat.clone().requires_grad_(True)
    ac = __import__("copy").deepcopy(mod)
    fc = feat.clone().requires_grad_(True)
    za = projection_head(fa, mod, wc)
    zr = ref(fr)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        zc = ac(fc).float()
    rel = lambda u, v: ((u.double() - v.double()).norm() / v.double().norm().clamp_min(1e-12)).item()  # noqa: E731
    # error budget: torch's own bf16 autocast of the same head against fp32 (the ReLU mask
    # flips at near-zero hidden units dominate the backward), with 1.5x slack and a floor
    env = lambda a, c, r: max(1.5 * rel(c, r), 4e-3)  # noqa: E731
    assert za.dtype == torch.float32 and za.shape == zr.shape
    assert rel(za, zr) < env(za, zc, zr), (rel(za, zr), rel(zc, zr))
    g = torch.randn_like(za)
    za.backward(g)
    zr.backward(g)
    zc.backward(g)
    assert rel(fa.grad, fr.grad) < env(fa.grad, fc.grad, fr.grad), (rel(fa.grad, fr.grad), rel(fc.grad, fr.grad))
    for (n, pa), pr, pc in zip(mod.named_parameters(), ref.parameters(), ac.parameters()):
        assert rel(pa.grad, pr.grad) < env(pa.grad, pc.grad, pr.grad), (n, rel(pa.grad, pr.grad), rel(pc.grad, pr.grad))
    # gradients accumulate into the sinks (a second backward doubles them)
    g1 = [p.grad.clone() for p in mod.parameters()]
    projection_head(feat.clone().requires_grad_(True), mod, wc).backward(g)
    for p, a in zip(mod.parameters(), g1):
        assert torch.allclose(p.grad, 2 * a, rtol=1e-5, atol=1e-6)
