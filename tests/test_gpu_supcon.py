"""Fused contrastive-loss kernel vs the fp64 torch oracle (GPU)."""
import pytest
import torch
import torch.nn.functional as F

from simclr_pytorch_distributed_amd.losses.supcon import supcon_rows_reference

pytestmark = pytest.mark.gpu


def _case(n_samples, D, n_views=2, supcon=False, mode="all", seed=0, dev="cuda"):
    g = torch.Generator().manual_seed(seed)
    C = F.normalize(torch.randn(n_views * n_samples, D, generator=g), dim=1)
    sample = torch.arange(n_samples).repeat(n_views)
    key = torch.randint(0, 7, (n_samples,), generator=g).repeat(n_views) if supcon else sample
    if mode == "all":
        self_idx = torch.arange(n_views * n_samples)
    else:
        self_idx = torch.arange(n_samples)
    return (C.to(dev), self_idx.to(torch.int32).to(dev), key.to(torch.int32).to(dev))


@pytest.mark.parametrize("n,D,supcon,mode", [
    (256, 128, False, "all"),   # README config, W=1
    (100, 128, False, "all"),   # ragged tiles
    (256, 128, True, "all"),
    (96, 64, True, "one"),
    (64, 256, False, "all"),
    (1024, 128, False, "all"),
])
def test_supcon_kernel_matches_oracle(gpu, n, D, supcon, mode):
    from simclr_pytorch_distributed_amd.ops.contrastive import supcon_rows_loss
    C, self_idx, key = _case(n, D, supcon=supcon, mode=mode)
    A_idx = self_idx.long()
    temp, base = 0.5, 0.07
    scale = 1.0 / A_idx.numel()

    Cn = C.clone().requires_grad_(True)
    A = Cn[A_idx]
    loss, rows = supcon_rows_loss(A, Cn, self_idx, key[A_idx], key, temp, base, scale, return_rows=True)
    (loss * 1.7).backward()

    Cr = C.double().clone().requires_grad_(True)
    Ar = Cr[A_idx]
    ref_rows = supcon_rows_reference(Ar, Cr, self_idx, key[A_idx], key, temp, base)
    ref = scale * ref_rows.sum()
    (ref * 1.7).backward()

    assert torch.allclose(rows.double(), ref_rows.detach(), rtol=1e-4, atol=1e-4), \
        (rows[:4], ref_rows[:4])
    assert abs(loss.item() - ref.item()) < 1e-4 * max(1.0, abs(ref.item()))
    err = (Cn.grad.double() - Cr.grad).abs().max().item()
    assert err < 1e-4 * Cr.grad.abs().max().item() + 1e-7, err


def test_supcon_golden_identical(gpu):
    from simclr_pytorch_distributed_amd.losses.supcon import SupConLoss
    f = F.normalize(torch.ones(256, 2, 128, device=gpu), dim=-1)
    loss = SupConLoss(temperature=0.5, backend="native")(f)
    assert abs(loss.item() - 44.5455) < 2e-3


@pytest.mark.parametrize("na,n", [(1024, 8192), (512, 512)])
def test_supcon_backward_deterministic(gpu, na, n):
    """Config-5 scale (1024 local anchors x 8192 gathered contrasts, SupCon keys): the
    backward writes per-split partial slabs summed in fixed order — bitwise identical
    gradients across runs (no atomics), and within fp32 tolerance of the fp64 oracle."""
    from simclr_pytorch_distributed_amd.ops import _ext
    ext = _ext.require()
    g = torch.Generator().manual_seed(5)
    C = F.normalize(torch.randn(n, 128, generator=g), dim=1).to(gpu)
    keys = torch.randint(0, 100, (n,), generator=g).to(torch.int32).to(gpu)
    self_idx = torch.arange(na, dtype=torch.int32, device=gpu)
    A = C[:na].contiguous()
    inv_t, ratio = 1 / 0.1, 0.1 / 0.07
    loss, lse, invcnt, rows = ext.supcon_fwd(A, C, self_idx, keys[:na].contiguous(), keys, inv_t, ratio, 1.0 / na)
    gs = torch.ones(1, device=gpu)
    outs = [ext.supcon_bwd(A, C, self_idx, keys[:na].contiguous(), keys, lse, invcnt, gs, inv_t, ratio * inv_t / na)
            for _ in range(3)]
    for dA, dC in outs[1:]:
        assert torch.equal(dA, outs[0][0]) and torch.equal(dC, outs[0][1])
    Cr = C.double().clone().requires_grad_(True)
    Ar = Cr[:na]
    ref = supcon_rows_reference(Ar, Cr, self_idx, keys[:na], keys, 0.1, 0.07).sum() / na
    ref.backward()
    got = outs[0][1].double()
    got[:na] += outs[0][0].double()
    err = (got - Cr.grad).abs().max().item()
    assert err < 1e-4 * Cr.grad.abs().max().item() + 1e-7, err


@pytest.mark.parametrize("n,D,supcon", [(256, 128, False), (100, 128, True), (2048, 128, False)])
def test_supcon_backward_sum_when_anchors_are_contrasts(gpu, n, D, supcon):
    """One rank, contrast_mode "all": the anchors ARE the contrast tensor, and the backward
    sums dA + dC inside its split reduction (supcon_bwd_sum) instead of a separate reduce +
    an autograd add. Same gradient as the two-output path (fp32 summation order aside) and
    as the fp64 oracle."""
    from simclr_pytorch_distributed_amd.ops.contrastive import supcon_rows_loss
    C, self_idx, key = _case(n, D, supcon=supcon, mode="all")
    temp, base = 0.5, 0.07
    scale = 1.0 / self_idx.numel()
    X = C.clone().requires_grad_(True)
    supcon_rows_loss(X, X, self_idx, key, key, temp, base, scale).backward()      # merged
    Y = C.clone().requires_grad_(True)
    supcon_rows_loss(Y * 1.0, Y, self_idx, key, key, temp, base, scale).backward()  # two outputs
    assert torch.allclose(X.grad, Y.grad, rtol=1e-5, atol=1e-7), (X.grad - Y.grad).abs().max()
    Cr = C.double().clone().requires_grad_(True)
    (scale * supcon_rows_reference(Cr, Cr, self_idx, key, key, temp, base).sum()).backward()
    err = (X.grad.double() - Cr.grad).abs().max().item()
    assert err < 1e-4 * Cr.grad.abs().max().item() + 1e-7, err
