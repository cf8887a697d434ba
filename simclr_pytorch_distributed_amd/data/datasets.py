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
    images: np.ndarray      # uint8 [N, H, W, 3]
    labels: np.ndarray      # int64 [N]
    num_classes: int
    name: str = ""

    def __len__(self):
        return int(self.images.shape[0])


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


def load_image_folder(root: str, size: Optional[int] = None) -> ArrayDataset:
    """ImageFolder (class-per-subdirectory) decoded with PIL into a uint8 array.

    Images are resized to ``size`` x ``size`` (if given) so the dataset can be stored as
    one dense array for the GPU augmentation kernel.
    """
    from PIL import Image
    classes = sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d)))
    exts = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")
    xs, ys = [], []
    for ci, cname in enumerate(classes):
        cdir = os.path.join(root, cname)
        for dp, _, files in sorted(os.walk(cdir)):
            for f in sorted(files):
                if f.lower().endswith(exts):
                    im = Image.open(os.path.join(dp, f)).convert("RGB")
                    if size is not None:
                        im = im.resize((size, size), Image.BILINEAR)
                    xs.append(np.asarray(im, dtype=np.uint8))
                    ys.append(ci)
    if not xs:
        raise FileNotFoundError(f"no images under {root!r}")
    return ArrayDataset(np.stack(xs), np.asarray(ys, dtype=np.int64), len(classes), os.path.basename(root))


def build_dataset(dataset: str, data_folder: str, train: bool = True, synthetic: bool = False,
                  synthetic_size: int = 50000, size: int = 32, seed: int = 0) -> ArrayDataset:
    if synthetic:
        ncls = {"cifar10": 10, "cifar100": 100}.get(dataset, 10)
        n = synthetic_size if train else max(1000, synthetic_size // 5)
        return synthetic_dataset(n, size if dataset == "path" else 32, ncls, seed + (0 if train else 1), class_seed=seed)
    if dataset in _CIFAR:
        return load_cifar(dataset, data_folder, train)
    if dataset == "path":
        return load_image_folder(data_folder, size)
    raise ValueError(f"dataset not supported: {dataset}")
