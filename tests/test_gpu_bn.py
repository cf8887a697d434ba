"""Fused BatchNorm kernels vs torch.batch_norm in fp32 (GPU)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("res_mode", [0, 1, 2])
def test_bn_train_fwd_bwd(gpu, res_mode):
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    torch.manual_seed(0)
    N, H, W, C = 16, 8, 8, 128
    y = (torch.randn(N, H, W, C, device=gpu) * 2 + 0.5).bfloat16()
    y2 = (torch.randn(N, H, W, C, device=gpu) - 1).bfloat16()
    g1 = torch.rand(C, device=gpu) + 0.5
    b1 = torch.randn(C, device=gpu)
    g2 = torch.rand(C, device=gpu) + 0.5
    b2 = torch.randn(C, device=gpu)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    rm2, rv2 = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)

    # reference in fp32 NCHW
    yf = y.float().permute(0, 3, 1, 2).requires_grad_(True)
    y2f = y2.float().permute(0, 3, 1, 2).requires_grad_(True)
    g1r, b1r, g2r, b2r = [t.clone().requires_grad_(True) for t in (g1, b1, g2, b2)]
    rmr, rvr = rm.clone(), rv.clone()
    o = F.batch_norm(yf, rmr, rvr, g1r, b1r, training=True, momentum=0.1, eps=1e-5)
    if res_mode == 1:
        o = o + F.batch_norm(y2f, rm2.clone(), rv2.clone(), g2r, b2r, training=True, momentum=0.1, eps=1e-5)
    elif res_mode == 2:
        o = o + y2f
    o = F.relu(o)
    dout = torch.randn(N, H, W, C, device=gpu).bfloat16()
    o.backward(dout.float().permute(0, 3, 1, 2))

    # native
    count = N * H * W
    flat = y.reshape(-1, C).float()
    sums = torch.stack([flat.sum(0), (flat * flat).sum(0)]).double().contiguous()
    sc, sh, mean, inv = m.bn_finalize(sums, float(count), g1, b1, 1e-5, 0.1, True, rm, rv)
    sc2 = sh2 = mean2 = inv2 = None
    if res_mode == 1:
        flat2 = y2.reshape(-1, C).float()
        sums2 = torch.stack([flat2.sum(0), (flat2 * flat2).sum(0)]).double().contiguous()
        sc2, sh2, mean2, inv2 = m.bn_finalize(sums2, float(count), g2, b2, 1e-5, 0.1, True, rm2, rv2)
    out = m.bn_apply(y, sc, sh, y2 if res_mode else None, sc2, sh2, res_mode, True)
    assert _rel(out.permute(0, 3, 1, 2), o.detach()) < 1e-2
    assert torch.allclose(rm, rmr, atol=1e-4) and torch.allclose(rv, rvr, rtol=1e-3)

    do = dout.contiguous()
    two = res_mode == 1
    s = m.bn_bwd_reduce(do, out, y, mean, y2 if two else None, mean2 if two else None)
    ca, cb, dga, dba, dgb, dbb = m.bn_bwd_coef(s, float(count), g1, mean, inv, g2 if two else None,
                                               mean2 if two else None, inv2 if two else None)
    dya, dyb, dz = m.bn_bwd_apply(do, out, y, ca, y2 if two else None, cb if two else None, res_mode == 2)
    assert _rel(dya.permute(0, 3, 1, 2), yf.grad) < 2e-2
    assert _rel(dga, g1r.grad) < 1e-2 and _rel(dba, b1r.grad) < 1e-2
    if two:
        assert _rel(dyb.permute(0, 3, 1, 2), y2f.grad) < 2e-2
        assert _rel(dgb, g2r.grad) < 1e-2 and _rel(dbb, b2r.grad) < 1e-2
    if res_mode == 2:
        assert _rel(dz.permute(0, 3, 1, 2), y2f.grad) < 1e-2


def test_bn_eval_affine(gpu):
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    C = 64
    rm, rv = torch.randn(C, device=gpu), torch.rand(C, device=gpu) + 0.1
    g, b = torch.randn(C, device=gpu), torch.randn(C, device=gpu)
    sc, sh = m.bn_eval_affine(g, b, rm, rv, 1e-5)
    y = torch.randn(4, 4, 4, C, device=gpu).bfloat16()
    out = m.bn_apply(y, sc, sh, None, None, None, 0, False)
    ref = F.batch_norm(y.float().permute(0, 3, 1, 2), rm, rv, g, b, training=False, eps=1e-5)
    assert _rel(out.permute(0, 3, 1, 2), ref) < 1e-2


def test_bn_bwd_mask_from_input(gpu):
    """bn_bwd_reduce/apply with the ReLU mask recomputed from y (msc/msh) == with the
    stored activation."""
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    torch.manual_seed(1)
    N, H, W, C = 8, 8, 8, 64
    y = (torch.randn(N, H, W, C, device=gpu) + 0.2).bfloat16()
    g1, b1 = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    flat = y.reshape(-1, C).float()
    sums = torch.stack([flat.sum(0), (flat * flat).sum(0)]).double().contiguous()
    sc, sh, mean, inv = m.bn_finalize(sums, float(N * H * W), g1, b1, 1e-5, 0.1, False, None, None)
    a = m.bn_apply(y, sc, sh, None, None, None, 0, True)
    dout = torch.randn(N, H, W, C, device=gpu).bfloat16()
    s_ref = m.bn_bwd_reduce(dout, a, y, mean)
    s = m.bn_bwd_reduce(dout, None, y, mean, msc=sc, msh=sh)
    assert torch.allclose(s, s_ref, rtol=1e-4, atol=1e-3)
    ca = m.bn_bwd_coef(s_ref, float(N * H * W), g1, mean, inv)[0]
    d_ref = m.bn_bwd_apply(dout, a, y, ca)[0]
    d = m.bn_bwd_apply(dout, None, y, ca, msc=sc, msh=sh)[0]
    assert _rel(d, d_ref) < 1e-2


@pytest.mark.parametrize("rows,C", [(1, 64), (37, 128), (4096, 64), (300, 2048)])
def test_single_launch_stats_finalize(gpu, rows, C):
    """bn_stats_finalize (one launch: per-block partials + last-arriver combine) ==
    bn_stats_reduce + bn_finalize == fp64 torch, bitwise-stable across repeated calls."""
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    torch.manual_seed(2)
    slab = torch.randn(rows, 2, C, device=gpu)
    slab[:, 1] = slab[:, 1].abs() * 3 + slab[:, 0] ** 2
    ref = slab.double().sum(0)
    s = m.bn_stats_reduce(slab)
    assert torch.allclose(s, ref, rtol=1e-12, atol=1e-9)
    g, b = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    count = float(rows * 16)
    rm1, rv1 = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    rm2, rv2 = rm1.clone(), rv1.clone()
    a = m.bn_finalize(s, count, g, b, 1e-5, 0.1, True, rm1, rv1)
    outs = [m.bn_stats_finalize(slab, count, g, b, 1e-5, 0.1, True, rm2, rv2)]
    for t, u in zip(a, outs[0]):
        assert torch.equal(t, u)
    assert torch.equal(rm1, rm2) and torch.equal(rv1, rv2)
    for _ in range(3):   # counters reset by the last block: repeated launches stay exact
        o = m.bn_stats_finalize(slab, count, g, b, 1e-5, 0.1, False, None, None)
        for t, u in zip(a, o):
            assert torch.equal(t, u)


@pytest.mark.parametrize("two", [False, True])
def test_bwd_reduce_coef_fused(gpu, two):
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    torch.manual_seed(3)
    N, H, W, C = 32, 16, 16, 64
    y = torch.randn(N, H, W, C, device=gpu).bfloat16()
    y2 = torch.randn(N, H, W, C, device=gpu).bfloat16()
    out = torch.relu(torch.randn(N, H, W, C, device=gpu)).bfloat16()
    dout = torch.randn(N, H, W, C, device=gpu).bfloat16()
    mu, inv = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    mu2, inv2 = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    g1, g2 = torch.rand(C, device=gpu) + 0.5, torch.rand(C, device=gpu) + 0.5
    cnt = float(N * H * W)
    yb, mb = (y2, mu2) if two else (None, None)
    s = m.bn_bwd_reduce(dout, out, y, mu, yb, mb)
    ref = m.bn_bwd_coef(s, cnt, g1, mu, inv, g2 if two else None, mb, inv2 if two else None)
    for _ in range(2):
        got = m.bn_bwd_reduce_coef(dout, out, y, mu, yb, mb, None, None, cnt, g1, inv, g2 if two else None,
                                   inv2 if two else None)
        for t, u in zip(ref, got):
            assert torch.equal(t, u)
    # sinks accumulate
    sga, sba = torch.ones(C, device=gpu), torch.ones(C, device=gpu)
    kw = dict(sink_ga=sga, sink_ba=sba)
    if two:
        kw.update(sink_gb=torch.ones(C, device=gpu), sink_bb=torch.ones(C, device=gpu))
    m.bn_bwd_reduce_coef(dout, out, y, mu, yb, mb, None, None, cnt, g1, inv, g2 if two else None,
                         inv2 if two else None, **kw)
    assert torch.allclose(sga, ref[2] + 1) and torch.allclose(sba, ref[3] + 1)


def test_relu_bitmask_matches_activation(gpu):
    """bn_apply(mask_out=) writes the ReLU bits of its output; the backward kernels give
    identical results from the bitmask and from the bf16 activation."""
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    torch.manual_seed(5)
    N, H, W, C = 4, 8, 8, 256
    y = torch.randn(N, H, W, C, device=gpu).bfloat16()
    r = torch.randn(N, H, W, C, device=gpu).bfloat16()
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    mask = torch.empty(y.numel() // 8, dtype=torch.uint8, device=gpu)
    out = m.bn_apply(y, sc, sh, r, None, None, 2, True, mask_out=mask)
    bits = ((mask.long().unsqueeze(1) >> torch.arange(8, device=gpu)) & 1).reshape(-1)
    assert torch.equal(bits.bool(), (out.reshape(-1).float() > 0))
    d = torch.randn_like(out)
    mu, iv = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    s1, s2 = m.bn_bwd_reduce(d, out, y, mu), m.bn_bwd_reduce(d, mask, y, mu)
    assert torch.equal(s1, s2)
    ca = m.bn_bwd_coef(s1, float(N * H * W), sc, mu, iv)[0]
    a1 = m.bn_bwd_apply(d, out, y, ca, None, None, True)
    a2 = m.bn_bwd_apply(d, mask, y, ca, None, None, True)
    assert torch.equal(a1[0], a2[0]) and torch.equal(a1[2], a2[2])
