"""Data pipeline parity (CPU): ImageFolder decoding at native resolution into the ragged
store (RandomResizedCrop samples the original pixels, main_supcon.py:170-191), the
resized dense store, the threaded decode (--num_workers), and the --gpu_aug 0 CPU path."""
import numpy as np
import pytest
import torch


def _folder(tmp_path, shapes):
    from PIL import Image
    rng = np.random.default_rng(0)
    out = []
    for i, (h, w) in enumerate(shapes):
        d = tmp_path / f"class{i % 2}"
        d.mkdir(exist_ok=True)
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        Image.fromarray(a).save(d / f"img{i:02d}.png")
        out.append((i % 2, a))
    return out


def test_image_folder_native_and_resized(tmp_path):
    from simclr_pytorch_distributed_amd.data.datasets import build_dataset
    shapes = [(40, 30), (17, 64), (33, 33), (64, 20), (25, 51)]
    src = _folder(tmp_path, shapes)
    ds = build_dataset("path", str(tmp_path), native=True, workers=3)
    assert ds.ragged and len(ds) == len(shapes) and ds.num_classes == 2
    by_class = sorted(src, key=lambda t: t[0])            # ImageFolder order: class, then file
    got = sorted((tuple(ds.image(i).shape), int(ds.labels[i])) for i in range(len(ds)))
    assert got == sorted((a.shape, c) for c, a in src)
    for i in range(len(ds)):
        assert any(np.array_equal(ds.image(i), a) for _, a in by_class)   # pixels bit-exact
    dense = build_dataset("path", str(tmp_path), size=16, workers=2)
    assert not dense.ragged and dense.images.shape == (len(shapes), 16, 16, 3)


def test_image_folder_side_cap_and_budget(tmp_path):
    """The ragged store caps the shorter side at ragged_side_cap(size) (aspect kept); over
    the byte budget it lowers that cap (still ragged, aspect ratios kept: RandomResizedCrop
    keeps sampling the native geometry) and raises when even a cap at the crop size does not
    fit (no silent squashed square store)."""
    from simclr_pytorch_distributed_amd.data.datasets import load_image_folder, ragged_side_cap
    assert ragged_side_cap(32) == 83 and ragged_side_cap(224) == 579
    _folder(tmp_path, [(120, 60), (40, 200), (30, 30)])
    ds = load_image_folder(str(tmp_path), None, 2, max_side=50)
    hw = sorted(tuple(int(v) for v in s) for s in ds.sizes)
    assert hw == sorted([(100, 50), (40, 200), (30, 30)])
    assert ds.images.size == sum(h * w * 3 for h, w in hw)
    small = load_image_folder(str(tmp_path), None, 2, max_side=50, budget_bytes=20000, dense_size=16)
    assert small.ragged and small.images.size <= 20000
    hw2 = sorted(tuple(int(v) for v in s) for s in small.sizes)
    assert hw2 == sorted([(56, 28), (28, 140), (28, 28)])       # shorter sides capped at 28
    for (h, w), (h2, w2) in zip(hw, hw2):
        assert abs(h / w - h2 / w2) < 0.05 * (h / w)
    with pytest.raises(RuntimeError, match="SDX_DATA_BUDGET_GB"):
        load_image_folder(str(tmp_path), None, 2, max_side=50, budget_bytes=1000, dense_size=16)


def test_ragged_reference_augment_matches_dense():
    """Same-size images: the ragged CPU path reproduces the dense one exactly."""
    from simclr_pytorch_distributed_amd.data.augment import AugConfig, augment_reference
    g = torch.Generator().manual_seed(0)
    data = torch.randint(0, 256, (6, 20, 28, 3), generator=g, dtype=torch.uint8)
    offs = torch.arange(6, dtype=torch.int64) * 20 * 28 * 3
    hw = torch.tensor([[20, 28]] * 6, dtype=torch.int32)
    idx = torch.tensor([4, 1, 5, 0])
    cfg = AugConfig.simclr(16, (0.5, 0.5, 0.5), (0.25, 0.25, 0.25))
    a = augment_reference(data, idx, cfg, 3)
    b = augment_reference(data.reshape(-1), idx, cfg, 3, offs, hw)
    assert torch.equal(a, b)


@pytest.mark.parametrize("gpu_aug", [0])
def test_engine_step_image_folder_cpu_aug(tmp_path, gpu_aug):
    """dataset=path at native resolutions through the engine with --gpu_aug 0 (torch CPU)."""
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    (tmp_path / "data").mkdir()
    _folder(tmp_path / "data", [(40, 30), (17, 64), (33, 33), (64, 20), (25, 51), (36, 36), (28, 40), (50, 22)])
    opt = parse_pretrain(["--model", "resnet18", "--backend", "torch", "--dataset", "path", "--data_folder",
                          str(tmp_path / "data"), "--mean", "(0.5,0.5,0.5)", "--std", "(0.25,0.25,0.25)",
                          "--size", "16", "--batch_size", "4", "--gpu_aug", str(gpu_aug), "--num_workers", "2",
                          "--work_dir", str(tmp_path / "ws")], make_dirs=False)
    eng = PretrainEngine(opt)
    assert eng.data_offs is not None and eng.data.dim() == 1
    st = eng.train_step(torch.arange(4), 1, 0, 2)
    assert torch.isfinite(st["loss_local"])


def test_two_crop_transform_gives_two_distinct_views():
    """TwoCropTransform(SimCLRAugment) (reference util.py:10-16 with the SimCLR pipeline):
    two normalized [3, S, S] views of one uint8 image, drawn independently."""
    from simclr_pytorch_distributed_amd.data.augment import AugConfig, SimCLRAugment, TwoCropTransform
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (40, 40, 3), dtype=torch.uint8, generator=g)
    t = TwoCropTransform(SimCLRAugment(AugConfig(size=32), seed=3))
    v1, v2 = t(img)
    assert v1.shape == v2.shape == (3, 32, 32) and v1.dtype == torch.float32
    assert not torch.equal(v1, v2)
    assert torch.isfinite(v1).all() and torch.isfinite(v2).all()
