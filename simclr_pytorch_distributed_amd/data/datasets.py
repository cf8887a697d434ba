"""In-memory datasets: CIFAR-10/100 (both the python-pickle and the binary release
formats), synthetic CIFAR-shaped data, and an ImageFolder reader.

Replaces torchvision.datasets.CIFAR10/CIFAR100/ImageFolder used by the reference
(main_supcon.py:181-193, main_ce.py:42-58). The MI355X design keeps the whole uint8
dataset resident in HBM (CIFAR-10 train = 150 MiB of 288 GB) and augments on the GPU,
so a dataset here is just ``images: uint8 [N, H, W, 3]`` + ``labels: int64 [N]``.

No download: there is no network. ``download=True`` semantics of the reference are
replaced by a clear error naming the expected files.
"""
from __future__ import annotations

import os
import pickle
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np


@dataclass
class ArrayDataset:
    images: np.ndarray      # uint8 [N, H, W, 3], or a flat uint8 byte store (ragged)
    labels: np.ndarray      # int64 [N]
    num_classes: int
    name: str = ""
    # ragged store of native-resolution images: image i is images[offsets[i]:][:h*w*3]
    # with (h, w) = sizes[i] (int64 [N] / int32 [N, 2]); None for a dense store
    offsets: Optional[np.ndarray] = None
    sizes: Optional[np.ndarray] = None

    def __len__(self):
        return int(self.labels.shape[0])

    @property
    def ragged(self) -> bool:
        return self.offsets is not None

    def image(self, i: int) -> np.ndarray:
        """Image i as uint8 [h, w, 3] (either store)."""
        if not self.ragged:
            return self.images[i]
        h, w = (int(v) for v in self.sizes[i])
        o = int(self.offsets[i])
        return self.images[o:o + h * w * 3].reshape(h, w, 3)


_CIFAR = {
    "cifar10": dict(py="cifar-10-batches-py", bin="cifar-10-batches-bin",
                    train=[f"data_batch_{i}" for i in range(1, 6)], test=["test_batch"],
                    bin_train=[f"data_batch_{i}.bin" for i in range(1, 6)], bin_test=["test_batch.bin"],
                    label_key="labels", label_bytes=1, ncls=10),
    "cifar100": dict(py="cifar-100-python", bin="cifar-100-binary", train=["train"], test=["test"],
                     bin_train=["train.bin"], bin_test=["test.bin"], label_key="fine_labels", label_bytes=2,
                     ncls=100),
}


def _load_py_batches(folder: str, files, label_key: str) -> Tuple[np.ndarray, np.ndarray]:
    # The CIFAR python release is a pickle of plain dicts of numpy arrays (user data, not
    # reference-shipped files).
    xs, ys = [], []
    for f in files:
        with open(os.path.join(folder, f), "rb") as fh:
            d = pickle.load(fh, encoding="latin1")
        xs.append(np.asarray(d["data"], dtype=np.uint8))
        ys.append(np.asarray(d[label_key], dtype=np.int64))
    x = np.concatenate(xs).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(x), np.concatenate(ys)


def _load_bin_batches(folder: str, files, label_bytes: int) -> Tuple[np.ndarray, np.ndarray]:
    xs, ys = [], []
    rec = label_bytes + 3072
    for f in files:
        raw = np.fromfile(os.path.join(folder, f), dtype=np.uint8)
        raw = raw.reshape(-1, rec)
        ys.append(raw[:, label_bytes - 1].astype(np.int64))   # cifar100: [coarse, fine]
        xs.append(raw[:, label_bytes:])
    x = np.concatenate(xs).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(x), np.concatenate(ys)


def load_cifar(name: str, root: str, train: bool = True) -> ArrayDataset:
    spec = _CIFAR[name]
    py_dir = os.path.join(root, spec["py"])
    bin_dir = os.path.join(root, spec["bin"])
    if os.path.isdir(py_dir):
        x, y = _load_py_batches(py_dir, spec["train"] if train else spec["test"], spec["label_key"])
    elif os.path.isdir(bin_dir):
        x, y = _load_bin_batches(bin_dir, spec["bin_train"] if train else spec["bin_test"], spec["label_bytes"])
    else:
        raise FileNotFoundError(
            f"{name} not found under {root!r}: expected {spec['py']}/ or {spec['bin']}/ "
            "(no network here: place the dataset there, or use --synthetic)")
    return ArrayDataset(x, y, spec["ncls"], name)


def synthetic_dataset(n: int = 50000, size: int = 32, num_classes: int = 10, seed: int = 0,
                      class_seed: int = 0) -> ArrayDataset:
    """CIFAR-shaped random images with class-dependent colour/texture statistics, so a
    linear probe on learned features has a signal (plumbing/accuracy smoke tests).
    The per-class statistics come from ``class_seed`` (shared by the train and validation
    splits); ``seed`` draws the labels and the per-image noise."""
    crng = np.random.default_rng(1_000_003 + class_seed)
    base = crng.integers(30, 225, size=(num_classes, 1, 1, 3))
    freq = crng.uniform(0.2, 1.2, size=(num_classes,))
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, num_classes, size=n).astype(np.int64)
    yy, xx = np.mgrid[0:size, 0:size]
    imgs = np.empty((n, size, size, 3), dtype=np.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        lab = labels[s:s + chunk]
        pat = np.sin(freq[lab][:, None, None] * (xx[None] + yy[None]))[..., None] * 40
        noise = rng.normal(0, 25, size=(lab.shape[0], size, size, 3))
        v = base[lab] + pat + noise
        imgs[s:s + chunk] = np.clip(v, 0, 255).astype(np.uint8)
    return ArrayDataset(imgs, labels, num_classes, "synthetic")


def ragged_side_cap(size: int, min_scale: float = 0.2, min_ratio: float = 3 / 4) -> int:
    """Shorter-side bound for the native-resolution store: RandomResizedCrop's smallest box
    (area ``min_scale``·H·W at aspect ``min_ratio``) still spans ``size`` source pixels
    when the shorter side is at most ``size / sqrt(min_scale·min_ratio)`` (≈2.58·size), so
    keeping more pixels than that adds bytes but no detail to any crop."""
    import math
    return int(math.ceil(size / math.sqrt(min_scale * min_ratio)))


def fit_ragged_budget(sizes: np.ndarray, budget: int, min_side: int = 1):
    """Shrink a ragged store's per-image (h, w) so its bytes fit ``budget``: every shorter
    side above a common cap is scaled down to it, aspect ratio kept (RandomResizedCrop then
    still samples its boxes from the native geometry, unlike a squashed square store). The
    cap starts at cap·sqrt(budget/total) and is lowered until the store fits; it never goes
    below ``min_side`` (the crop output size) — a folder that does not fit even then raises
    instead of silently degrading the augmentation. Returns (sizes, cap or None)."""
    import math
    sizes = np.asarray(sizes, dtype=np.int32).reshape(-1, 2)

    def total_of(sz):
        return int((sz[:, 0].astype(np.int64) * sz[:, 1] * 3).sum())

    total = total_of(sizes)
    if total <= budget:
        return sizes, None
    short = sizes.min(axis=1).astype(np.float64)
    cap = int(math.floor(short.max() * math.sqrt(budget / total)))
    while True:
        cap = max(int(min_side), cap)
        f = np.minimum(1.0, cap / np.maximum(short, 1.0))
        out = np.stack([np.maximum(1, np.round(sizes[:, 0] * f)), np.maximum(1, np.round(sizes[:, 1] * f))],
                       axis=1).astype(np.int32)
        if total_of(out) <= budget:
            return out, cap
        if cap <= min_side:
            raise RuntimeError(
                f"image store needs {total_of(out) / 2**30:.1f} GiB even with shorter sides capped at "
                f"{cap} px (> budget {budget / 2**30:.1f} GiB): raise SDX_DATA_BUDGET_GB")
        cap = int(cap * 0.97)


DATA_BUDGET_BYTES = int(float(os.environ.get("SDX_DATA_BUDGET_GB", "64")) * (1 << 30))


def load_image_folder(root: str, size: Optional[int] = None, workers: int = 1, max_side: Optional[int] = None,
                      budget_bytes: Optional[int] = None, dense_size: Optional[int] = None) -> ArrayDataset:
    """ImageFolder (class-per-subdirectory) decoded with PIL into uint8 RGB.

    ``size=None`` (pretraining): images are kept near their NATIVE resolution in a ragged
    byte store (offsets + sizes), so the GPU RandomResizedCrop samples its box from the
    original pixels as torchvision does on the decoded image (main_supcon.py:170-191).
    The shorter side is capped at ``max_side`` (aspect kept; see :func:`ragged_side_cap`),
    the sizes are read from the headers first and the flat store is preallocated and
    filled in place (no second copy). If the store would exceed ``budget_bytes`` (default
    ``SDX_DATA_BUDGET_GB``, 64 GiB: it lives in HBM next to training) the shorter-side cap
    is lowered until it fits (:func:`fit_ragged_budget`; aspect ratios kept, never below
    ``dense_size``), or a RuntimeError asks for a larger budget. ``size=s``: resized to s x s into a
    dense [N, s, s, 3] array. Decoding runs on ``workers`` threads (``--num_workers``; PIL
    releases the GIL while decoding).
    """
    import logging
    from concurrent.futures import ThreadPoolExecutor

    from PIL import Image
    classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
    exts = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")
    files, ys = [], []
    for ci, cname in enumerate(classes):
        cdir = os.path.join(root, cname)
        for dp, _, fs in sorted(os.walk(cdir)):
            for f in sorted(fs):
                if f.lower().endswith(exts):
                    files.append(os.path.join(dp, f))
                    ys.append(ci)
    if not files:
        raise FileNotFoundError(f"no images under {root!r}")
    labels = np.asarray(ys, dtype=np.int64)
    name = os.path.basename(os.path.normpath(root))
    nw = max(1, int(workers))

    def decode(path, hw=None):
        with Image.open(path) as im:
            im = im.convert("RGB")
            if hw is not None and (im.height, im.width) != hw:
                im = im.resize((hw[1], hw[0]), Image.BILINEAR)
            return np.asarray(im, dtype=np.uint8)

    def dense(s):
        out = np.empty((len(files), s, s, 3), dtype=np.uint8)

        def fill(i):
            out[i] = decode(files[i], (s, s))
        with ThreadPoolExecutor(max_workers=nw) as ex:
            list(ex.map(fill, range(len(files))))
        return ArrayDataset(out, labels, len(classes), name)

    if size is not None:
        return dense(size)

    def header(path):
        with Image.open(path) as im:          # lazy: reads the header only
            w, h = im.size
        if max_side is not None and min(h, w) > max_side:
            f = max_side / min(h, w)
            h, w = max(1, round(h * f)), max(1, round(w * f))
        return h, w

    with ThreadPoolExecutor(max_workers=nw) as ex:
        sizes = np.asarray(list(ex.map(header, files)), dtype=np.int32).reshape(-1, 2)
    budget = DATA_BUDGET_BYTES if budget_bytes is None else int(budget_bytes)
    sizes, cap = fit_ragged_budget(sizes, budget, min_side=dense_size or 1)
    if cap is not None:
        logging.warning(f"native-resolution store of {root!r} exceeds the {budget / 2**30:.1f} GiB budget: "
                        f"shorter sides capped at {cap} px (aspect kept; raise SDX_DATA_BUDGET_GB to keep more)")
    nbytes = sizes[:, 0].astype(np.int64) * sizes[:, 1] * 3
    total = int(nbytes.sum())
    offsets = np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(np.int64)
    flat = np.empty(total, dtype=np.uint8)

    def fill_ragged(i):
        h, w = (int(v) for v in sizes[i])
        o = int(offsets[i])
        flat[o:o + h * w * 3] = decode(files[i], (h, w)).reshape(-1)
    with ThreadPoolExecutor(max_workers=nw) as ex:
        list(ex.map(fill_ragged, range(len(files))))
    return ArrayDataset(flat, labels, len(classes), name, offsets=offsets, sizes=sizes)


def build_dataset(dataset: str, data_folder: str, train: bool = True, synthetic: bool = False,
                  synthetic_size: int = 50000, size: int = 32, seed: int = 0, native: bool = False,
                  workers: int = 1) -> ArrayDataset:
    """``native``: an ImageFolder (``dataset='path'``) keeps native resolutions (ragged
    store) for RandomResizedCrop; otherwise it is resized to ``size``."""
    if synthetic:
        ncls = {"cifar10": 10, "cifar100": 100}.get(dataset, 10)
        n = synthetic_size if train else max(1000, synthetic_size // 5)
        return synthetic_dataset(n, size if dataset == "path" else 32, ncls, seed + (0 if train else 1), class_seed=seed)
    if dataset in _CIFAR:
        return load_cifar(dataset, data_folder, train)
    if dataset == "path":
        if native:
            return load_image_folder(data_folder, None, workers, max_side=ragged_side_cap(size), dense_size=size)
        return load_image_folder(data_folder, size, workers)
    raise ValueError(f"dataset not supported: {dataset}")
