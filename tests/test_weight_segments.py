"""Weight-prep segment table (ops/weights.py, CPU): one row per conv / head Linear of the
flat fp32 master, each carrying the first 64x64-tap tile of its conv in the single flat
wprep grid (csrc/kernels/wprep.hip binary-searches it). The bit-exact GPU check of the
layouts is tests/test_gpu_misc.py::test_weight_cache_layouts_match_torch."""
import torch

from simclr_pytorch_distributed_amd.models.executor import INPUT_CHANNELS_PADDED
from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
from simclr_pytorch_distributed_amd.ops.weights import ConvWeightCache
from simclr_pytorch_distributed_amd.optim.flat import FlatParams


def test_segment_tiles_are_a_prefix_sum():
    m = SupConResNet("resnet50").to(memory_format=torch.channels_last)
    flat = FlatParams(m)
    convs = [mod for mod in m.modules() if isinstance(mod, (torch.nn.Conv2d, torch.nn.Linear))]
    wc = ConvWeightCache(convs, flat.flat, {id(m.encoder.conv1): INPUT_CHANNELS_PADDED})
    rows = wc.seg_rows
    assert len(rows) == len(convs)
    tile = 0
    for r, cv in zip(rows, convs):
        assert r[6] == tile
        K, C = r[3] & 0xffffffff, r[4] & 0xffffffff
        RS, Cp = r[3] >> 32, r[4] >> 32
        w = cv.weight
        assert (K, C) == (w.shape[0], w.shape[1]) and RS == (w.shape[2] * w.shape[3] if w.dim() == 4 else 1)
        assert Cp >= C and r[5] == K * RS * Cp
        tile += ((K + 63) // 64) * ((Cp + 63) // 64) * RS
    assert wc.tiles == tile
    # the largest conv alone set the old [largest x segments] grid: the flat grid is far smaller
    largest = max(((r[3] & 0xffffffff) + 63) // 64 * (((r[4] >> 32) + 63) // 64) * (r[3] >> 32) for r in rows)
    assert wc.tiles < largest * len(rows) / 4
