"""Tap-reuse 3x3 convolution loop (igemm.hip DEPTH 7 / 8, tile cfgs 11-13) vs fp32 torch (GPU).

The halo window of a tile (its image rows + the pad ring) is staged once per 64-channel chunk
and the 9 taps read it at uniform offsets; these tests cover every image width the loop is
built for (32 / 16 / 8 / 4: bands of one image, one image, 4 / 8 / 16 images per tile),
partial last tiles (batch not a multiple of the images per tile), output widths that are not
a multiple of the column tile, several channel chunks (the double-buffered halo), the
statistics epilogues (forward BN sums, dgrad BN-backward sums) and auto dispatch.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TAP_BM = {11: 256, 12: 256, 13: 128}
HALO_KB = {256: 50, 128: 36}


def tap_geom(cfg, H, W, cdim):
    """Python mirror of igemm.hip tap_geom: None if the tap cfg rejects the geometry, else the
    virtual row width of a padded-row tile (0: unpadded)."""
    bm = TAP_BM[cfg]
    if cdim % 64:
        return None
    hw = H * W
    rw = 0
    if bm % W or not (hw % bm == 0 or bm % hw == 0):
        rw = 16
        while rw < W:
            rw *= 2
        if cfg != 11 or bm % rw or H % (bm // rw):   # padded rows: the DEPTH-8 tile only
            return None
    imgs = bm // hw if (rw == 0 and bm >= hw) else 0
    rows = H if imgs > 0 else bm // (rw or W)
    hp = max(imgs, 1) * (rows + 2) * (W + 2)
    if math.ceil(hp / 8) > HALO_KB[bm]:
        return None
    if rw and (rows + 1) * (W + 2) + rw + 2 > HALO_KB[bm] * 8:
        return None
    if cfg == 11 and cdim != 64:
        return None
    return rw


def tap_ok(cfg, H, W, cdim):
    return tap_geom(cfg, H, W, cdim) is not None


def tap_mtiles(cfg, N, H, W, cdim):
    """statistics-slab rows: a padded-row tile counts its virtual rows"""
    bm, rw = TAP_BM[cfg], tap_geom(cfg, H, W, cdim)
    return N * H * rw // bm if rw else (N * H * W + bm - 1) // bm


# (N, H=W, C, K)
SHAPES = [
    (3, 32, 64, 64),     # layer-1 shape: bands of 8 (or 4) image rows
    (2, 32, 64, 96),     # output width not a multiple of the column tile
    (3, 16, 128, 128),   # one image per 256-row tile, 2 channel chunks
    (2, 16, 64, 192),
    (5, 8, 256, 256),    # 4 images per 256-row tile: the last tile holds one image
    (3, 8, 128, 64),
    (3, 4, 512, 512),    # 8 images per 128-row tile, 8 channel chunks (4 halo buffer swaps)
    (5, 4, 64, 128),
    # padded rows (config 5 at 224x224, cfg 11 only): 56 -> 64-slot rows (bands of 4 rows)
    (2, 56, 64, 64),
    (1, 56, 64, 96),
    (2, 28, 128, 128),
    (2, 14, 64, 64),     # 16-slot rows do not band 14 rows: rejected
]


def _mk(N, H, C, K, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, C, H, H, generator=g).cuda().bfloat16()
    w = (torch.randn(K, C, 3, 3, generator=g) / (C * 9) ** 0.5).cuda().bfloat16()
    return x, w


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cfg", [11, 12, 13])
def test_tap3_fwd(gpu, shape, cfg):
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    N, H, C, K = shape
    x, w = _mk(N, H, C, K)
    xh = x.permute(0, 2, 3, 1).contiguous()
    wh = w.permute(0, 2, 3, 1).contiguous()
    if not tap_ok(cfg, H, H, C):
        with pytest.raises(RuntimeError):
            m.conv_fwd(xh, wh, 1, 1, True, cfg)
        return
    ref = F.conv2d(x.float(), w.float(), padding=1)
    y, slab = m.conv_fwd(xh, wh, 1, 1, True, cfg)
    assert slab.shape[0] == tap_mtiles(cfg, N, H, H, C)
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-2
    sums = m.bn_stats_reduce(slab)
    yf = ref.permute(0, 2, 3, 1).reshape(-1, K).double()
    assert torch.allclose(sums[0], yf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(sums[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)
    # deterministic: the same launch twice gives the same bits
    y2, slab2 = m.conv_fwd(xh, wh, 1, 1, True, cfg)
    assert torch.equal(y, y2) and torch.equal(slab, slab2)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("cfg", [11, 12, 13])
def test_tap3_dgrad(gpu, shape, cfg):
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    N, H, C, K = shape
    x, w = _mk(N, H, C, K)
    xf = x.float().requires_grad_(True)
    out = F.conv2d(xf, w.float(), padding=1)
    dy = torch.randn_like(out).bfloat16()
    (dx_ref,) = torch.autograd.grad(out, xf, dy.float())
    wt = w.permute(1, 2, 3, 0).contiguous()            # [C][R][S][K]
    dyh = dy.permute(0, 2, 3, 1).contiguous()
    if not tap_ok(cfg, H, H, K):
        with pytest.raises(RuntimeError):
            m.conv_dgrad(dyh, wt, H, H, 1, 1, cfg)
        return
    dx = m.conv_dgrad(dyh, wt, H, H, 1, 1, cfg)
    assert _rel(dx.permute(0, 3, 1, 2), dx_ref) < 1e-2
    # with a residual addend (fused into the epilogue)
    add = torch.randn_like(dx)
    dx2 = m.conv_dgrad(dyh, wt, H, H, 1, 1, cfg, None, add)
    assert _rel(dx2.float(), dx.float() + add.float()) < 2e-2


@pytest.mark.parametrize("shape", [(3, 32, 64, 64), (3, 16, 128, 128), (5, 8, 256, 256), (3, 4, 512, 512),
                                   (2, 56, 64, 64)])
def test_tap3_dgrad_bnstat(gpu, shape):
    """dgrad + fused BN-backward statistics on the tap-reuse tiles (auto dispatch) against
    the same epilogue on the implicit-GEMM tile (cfg 4): equal statistics up to fp32
    summation order, the same dx up to bf16 rounding."""
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    N, H, C, K = shape
    x, w = _mk(N, H, C, K, seed=1)
    dy = torch.randn(N, H, H, K, device="cuda").bfloat16()
    wt = w.permute(1, 2, 3, 0).contiguous()
    ya = torch.randn(N, H, H, C, device="cuda").bfloat16()
    ma = torch.randn(C, device="cuda")
    bits = torch.randint(0, 256, (N * H * H * C // 8,), device="cuda", dtype=torch.uint8)
    outs = {}
    for cfg in (-1, 4):
        dx, slab = m.conv_dgrad_bnstat(dy, wt, H, H, 1, 1, cfg, None, None, None, ya, ma, None, None, bits,
                                       None, None)
        outs[cfg] = (dx, m.bn_stats_reduce(slab) if slab.shape[1] == 2 else None, slab)
    assert _rel(outs[-1][0], outs[4][0]) < 1e-2
    s_tap = outs[-1][2].double().sum(0)
    s_ref = outs[4][2].double().sum(0)
    assert torch.allclose(s_tap, s_ref, rtol=1e-3, atol=1e-1)


def _want(H, cdim, ncol):
    """the tap cfg auto dispatch picks (igemm_tap_cfg candidate order)"""
    for cfg in ([11] if cdim == 64 and ncol <= 64 else []) + ([12] if H >= 8 else []) + [13]:
        if tap_ok(cfg, H, H, cdim):
            return cfg
    return None


@pytest.mark.parametrize("shape", [(4, 32, 64, 64), (4, 16, 128, 128), (8, 8, 256, 256), (16, 4, 512, 512),
                                   (2, 56, 64, 64)])
def test_tap3_auto_dispatch(gpu, shape):
    """auto (cfg -1) runs the tap-reuse loop on every CIFAR ResNet 3x3 stride-1 shape and on
    the padded-row 56x56 stage of the 224x224 config."""
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    N, H, C, K = shape
    x, w = _mk(N, H, C, K, seed=2)
    xh = x.permute(0, 2, 3, 1).contiguous()
    wh = w.permute(0, 2, 3, 1).contiguous()
    want = _want(H, C, K)
    assert want is not None
    y_auto, s_auto = m.conv_fwd(xh, wh, 1, 1, True, -1)
    y_tap, s_tap = m.conv_fwd(xh, wh, 1, 1, True, want)
    assert torch.equal(y_auto, y_tap) and torch.equal(s_auto, s_tap)
    dy = torch.randn(N, H, H, K, device="cuda").bfloat16()
    wt = w.permute(1, 2, 3, 0).contiguous()
    want_d = _want(H, K, C)
    assert torch.equal(m.conv_dgrad(dy, wt, H, H, 1, 1, -1), m.conv_dgrad(dy, wt, H, H, 1, 1, want_d))
