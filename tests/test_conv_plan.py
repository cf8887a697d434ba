"""Conv dispatch plan (host-only, CPU): which tile config auto dispatch gives every stride-1
3x3 conv of the two benchmark configs, and how many statistics-slab rows its launch writes.

Covers the padded-row tap-reuse tiles (igemm.hip tap_geom t_rw): at 56x56 (224x224 config,
stage 1) a 256-row tile holds 4 image rows of 64 virtual pixels (56 real), so the slab has
N*H*64/256 rows, not ceil(N*H*W/256). The plan is computed by the extension's host code
only (`conv_plan`), no kernel runs.
"""
import pytest

from simclr_pytorch_distributed_amd.ops import _ext


@pytest.fixture(scope="module")
def m():
    mod = _ext.ext()
    if mod is None or not hasattr(mod, "conv_plan"):
        pytest.skip("native extension not built")
    return mod


# (N, H, C, K) -> expected tap cfg of the fwd and of the dgrad (both stride-1 3x3, pad 1)
CIFAR = [
    ((512, 32, 64, 64), 11),     # bands of 8 image rows
    ((512, 16, 128, 128), 12),   # one image per 256-row tile
    ((512, 8, 256, 256), 12),    # 4 images per tile
    ((512, 4, 512, 512), 13),    # 8 images per 128-row tile
]


@pytest.mark.parametrize("shape,cfg", CIFAR)
def test_cifar_3x3_on_tap_tiles(m, shape, cfg):
    N, H, C, K = shape
    bm = {11: 256, 12: 256, 13: 128}[cfg]
    for dgrad in (False, True):
        got_cfg, mt = m.conv_plan(N, H, H, C, K, 3, 3, 1, 1, dgrad)
        assert got_cfg == cfg
        assert mt == (N * H * H + bm - 1) // bm   # unpadded: whole images / bands


def test_56x56_padded_rows(m):
    N = 1024
    for dgrad in (False, True):
        cfg, mt = m.conv_plan(N, 56, 56, 64, 64, 3, 3, 1, 1, dgrad)
        assert cfg == 11
        assert mt == N * 56 * 64 // 256            # virtual rows: 64 per image row
        assert mt != (N * 56 * 56 + 255) // 256


@pytest.mark.parametrize("H,C", [(28, 128), (14, 256), (7, 512)])
def test_no_tap_tile_where_it_loses_or_misfits(m, H, C):
    # 28x28: the padded 128-row tile loses to the implicit GEMM (profiles/tap_pad_r6.txt);
    # 14x14 / 7x7: no band of whole (padded) rows fits a tile
    cfg, mt = m.conv_plan(1024, H, H, C, C, 3, 3, 1, 1, False)
    assert cfg not in (11, 12, 13)
    bm = {0: 128, 1: 256, 2: 64, 3: 64, 4: 128, 5: 256, 6: 128}[cfg]
    assert mt == (1024 * H * H + bm - 1) // bm


def test_1x1_plan_is_implicit_gemm(m):
    cfg, mt = m.conv_plan(512, 32, 32, 256, 64, 1, 1, 1, 0, False)
    assert cfg not in (11, 12, 13) and mt > 0
