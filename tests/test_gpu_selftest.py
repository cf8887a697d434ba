"""MFMA lane-map self test (asymmetric operands) on the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_mfma16_layout(gpu):
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    A = torch.arange(16 * 32, device=gpu, dtype=torch.float32).reshape(16, 32).remainder(7).sub(3).bfloat16()
    B = torch.arange(32 * 16, device=gpu, dtype=torch.float32).reshape(32, 16).remainder(5).sub(2).bfloat16()
    C = m.mfma16_selftest(A, B)
    assert torch.equal(C, A.float() @ B.float())
