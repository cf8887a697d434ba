"""SimCLR / linear-probe augmentation front-end.

GPU path: ``csrc/kernels/aug.hip`` — the reference's torchvision pipeline
(main_supcon.py:170-179 pretraining; main_ce.py:30-40 linear probe) fused into one
kernel over the HBM-resident uint8 dataset, writing NHWC bf16 (C padded to 8).

CPU path: :func:`augment_reference` — the same pipeline with the *same* counter-based
random draws, in torch (CPU runs, and the oracle the GPU kernel is tested against).
"""
from __future__ import annotations

import math
import dataclasses
from dataclasses import dataclass
from typing import Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..ops import _ext

M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


class _Rng:
    def __init__(self, key: int):
        self.key, self.ctr = key, 0

    def uni(self) -> float:
        v = _mix64(self.key ^ _mix64((0x1234567 + self.ctr) & M64))
        self.ctr += 1
        return float(np.float32((v >> 40) * (1.0 / 16777216.0)))


@dataclass
class AugConfig:
    size: int = 32
    n_views: int = 2
    scale: Sequence[float] = (0.2, 1.0)
    ratio: Sequence[float] = (3 / 4, 4 / 3)
    jitter_p: float = 0.8
    brightness: float = 0.4
    contrast: float = 0.4
    saturation: float = 0.4
    hue: float = 0.1
    gray_p: float = 0.2
    crop: bool = True
    flip: bool = True
    mean: Sequence[float] = (0.4914, 0.4822, 0.4465)
    std: Sequence[float] = (0.2023, 0.1994, 0.2010)

    @staticmethod
    def simclr(size, mean, std):
        return AugConfig(size=size, mean=mean, std=std)

    @staticmethod
    def linear_train(size, mean, std):
        # main_ce.py:30-35: RandomResizedCrop(32, scale=(0.2, 1)) + flip + normalize
        return AugConfig(size=size, n_views=1, jitter_p=0.0, brightness=0, contrast=0, saturation=0, hue=0,
                         gray_p=0.0, mean=mean, std=std)

    @staticmethod
    def evaluation(size, mean, std):
        # main_ce.py:37-40: ToTensor + normalize
        return AugConfig(size=size, n_views=1, jitter_p=0.0, brightness=0, contrast=0, saturation=0, hue=0,
                         gray_p=0.0, crop=False, flip=False, mean=mean, std=std)


def gpu_augment(data: torch.Tensor, idx: torch.Tensor, cfg: AugConfig, seed, seed_t=None, offs=None,
                hw=None) -> torch.Tensor:
    """``seed_t``: optional int64 device scalar read by the kernel at run time (graph replays).
    ``offs``/``hw``: a ragged native-resolution store (``data`` flat uint8, int64 byte
    offsets, int32 [N, 2] sizes; data/datasets.py load_image_folder)."""
    m = _ext.require()
    return m.gpu_augment(data, idx, cfg.size, cfg.n_views, int(seed) & ((1 << 63) - 1), list(cfg.mean),
                         list(cfg.std), cfg.scale[0], cfg.scale[1], cfg.ratio[0], cfg.ratio[1], cfg.jitter_p,
                         cfg.brightness, cfg.contrast, cfg.saturation, cfg.hue, cfg.gray_p, cfg.crop, cfg.flip,
                         seed_t, offs, hw)


def _view_params(cfg: AugConfig, H: int, W: int, rng: _Rng):
    f32 = np.float32
    ci, cj, ch, cw = 0.0, 0.0, float(H), float(W)
    if cfg.crop:
        area = f32(H) * f32(W)
        lr0, lr1 = f32(math.log(cfg.ratio[0])), f32(math.log(cfg.ratio[1]))
        found = False
        for _ in range(10):
            target = area * (f32(cfg.scale[0]) + (f32(cfg.scale[1]) - f32(cfg.scale[0])) * f32(rng.uni()))
            ar = f32(math.exp(lr0 + (lr1 - lr0) * f32(rng.uni())))
            w = float(np.rint(f32(math.sqrt(target * ar))))
            h = float(np.rint(f32(math.sqrt(target / ar))))
            if 0 < w <= W and 0 < h <= H:
                ci = math.floor(rng.uni() * (H - h + 1.0))
                cj = math.floor(rng.uni() * (W - w + 1.0))
                ch, cw = h, w
                found = True
                break
        if not found:
            in_ratio = W / H
            if in_ratio < cfg.ratio[0]:
                w, h = W, round(W / cfg.ratio[0])
            elif in_ratio > cfg.ratio[1]:
                h, w = H, round(H * cfg.ratio[1])
            else:
                w, h = W, H
            ci, cj, ch, cw = math.floor((H - h) * 0.5), math.floor((W - w) * 0.5), float(h), float(w)
    flip = cfg.flip and rng.uni() < 0.5
    jitter = rng.uni() < cfg.jitter_p
    fb = 1 + cfg.brightness * (2 * rng.uni() - 1)
    fc = 1 + cfg.contrast * (2 * rng.uni() - 1)
    fs = 1 + cfg.saturation * (2 * rng.uni() - 1)
    fh = cfg.hue * (2 * rng.uni() - 1)
    order = [0, 1, 2, 3]
    for i in range(3, 0, -1):
        j = int(rng.uni() * (i + 1)) % (i + 1)
        order[i], order[j] = order[j], order[i]
    gray = rng.uni() < cfg.gray_p
    if cfg.brightness <= 0 and cfg.contrast <= 0 and cfg.saturation <= 0 and cfg.hue <= 0:
        jitter = False
    return dict(ci=ci, cj=cj, ch=ch, cw=cw, flip=flip, jitter=jitter, fb=fb, fc=fc, fs=fs, fh=fh, order=order,
                gray=gray)


def _grey(img):
    return 0.2989 * img[0] + 0.587 * img[1] + 0.114 * img[2]


def _hue(img, hf):
    r, g, b = img[0], img[1], img[2]
    mx = torch.maximum(r, torch.maximum(g, b))
    mn = torch.minimum(r, torch.minimum(g, b))
    cr = mx - mn
    v = mx
    s = cr / torch.where(mx == 0, torch.ones_like(mx), mx)
    crd = torch.where(cr == 0, torch.ones_like(cr), cr)
    rc, gc, bc = (mx - r) / crd, (mx - g) / crd, (mx - b) / crd
    h = torch.where(mx == r, bc - gc, torch.where(mx == g, 2.0 + rc - bc, 4.0 + gc - rc))
    h = h / 6.0 + 1.0
    h = h - torch.floor(h)
    h = h + hf
    h = h - torch.floor(h)
    h6 = h * 6.0
    i = torch.floor(h6)
    f = h6 - i
    p = (v * (1 - s)).clamp(0, 1)
    q = (v * (1 - s * f)).clamp(0, 1)
    t = (v * (1 - s * (1 - f))).clamp(0, 1)
    i = i.long() % 6
    rr = torch.stack([v, q, p, p, t, v])
    gg = torch.stack([t, v, v, q, p, p])
    bb = torch.stack([p, p, t, v, v, q])
    sel = i.unsqueeze(0)
    return torch.stack([rr.gather(0, sel)[0], gg.gather(0, sel)[0], bb.gather(0, sel)[0]])


def augment_reference(data: torch.Tensor, idx: torch.Tensor, cfg: AugConfig, seed: int, offs=None,
                      hw=None) -> torch.Tensor:
    """CPU torch implementation with identical draws; returns NHWC float [V*B, S, S, 8]."""
    data = data.cpu()
    idx = idx.cpu()
    if offs is not None:
        offs, hw = offs.cpu(), hw.cpu()
    B = idx.shape[0]
    S = cfg.size
    seed = int(seed) & ((1 << 63) - 1)
    out = torch.zeros(cfg.n_views * B, S, S, 8)
    oy, ox = torch.meshgrid(torch.arange(S, dtype=torch.float32), torch.arange(S, dtype=torch.float32),
                            indexing="ij")
    for v in range(cfg.n_views):
        for b in range(B):
            src = int(idx[b])
            if offs is None:
                H, W = data.shape[1], data.shape[2]
                img = data[src].float()   # H W 3
            else:
                H, W = int(hw[src, 0]), int(hw[src, 1])
                o = int(offs[src])
                img = data[o:o + H * W * 3].view(H, W, 3).float()
            key = _mix64((seed * 0x100000001B3 + src * 31 + v * 0x9E37 + b) & M64)
            p = _view_params(cfg, H, W, _Rng(key))
            xs = (S - 1 - ox) if p["flip"] else ox
            sy = ((oy + 0.5) * (p["ch"] / S) - 0.5 + p["ci"]).clamp(p["ci"], p["ci"] + p["ch"] - 1)
            sx = ((xs + 0.5) * (p["cw"] / S) - 0.5 + p["cj"]).clamp(p["cj"], p["cj"] + p["cw"] - 1)
            y0, x0 = sy.floor().long(), sx.floor().long()
            y1, x1 = (y0 + 1).clamp(max=H - 1), (x0 + 1).clamp(max=W - 1)
            wy, wx = (sy - y0).unsqueeze(-1), (sx - x0).unsqueeze(-1)
            top = img[y0, x0] + (img[y0, x1] - img[y0, x0]) * wx
            bot = img[y1, x0] + (img[y1, x1] - img[y1, x0]) * wx
            c = ((top + (bot - top) * wy) / 255.0).permute(2, 0, 1)   # 3 S S
            if p["jitter"]:
                for op in p["order"]:
                    if op == 0:
                        c = (c * p["fb"]).clamp(0, 1)
                    elif op == 1:
                        mean = _grey(c).mean()
                        c = (p["fc"] * c + (1 - p["fc"]) * mean).clamp(0, 1)
                    elif op == 2:
                        g = _grey(c)
                        c = (p["fs"] * c + (1 - p["fs"]) * g).clamp(0, 1)
                    else:
                        c = _hue(c, p["fh"])
            if p["gray"]:
                c = _grey(c).unsqueeze(0).expand(3, S, S)
            mean_t = torch.tensor(cfg.mean).view(3, 1, 1)
            std_t = torch.tensor(cfg.std).view(3, 1, 1)
            c = (c - mean_t) / std_t
            out[v * B + b, :, :, :3] = c.permute(1, 2, 0)
    return out


def augment(data: torch.Tensor, idx: torch.Tensor, cfg: AugConfig, seed: int, offs=None, hw=None) -> torch.Tensor:
    """Dispatch: GPU kernel for GPU tensors, torch reference otherwise (NHWC, C=8)."""
    if data.is_cuda:
        return gpu_augment(data, idx, cfg, seed, offs=offs, hw=hw)
    return augment_reference(data, idx, cfg, seed, offs, hw)


def nhwc8_to_nchw(x: torch.Tensor) -> torch.Tensor:
    """NHWC [.., 8] -> NCHW float [.., 3, H, W] for the torch backend."""
    return x[..., :3].permute(0, 3, 1, 2).float().contiguous()


class SimCLRAugment:
    """Per-sample callable form of the SimCLR augmentation (reference main_supcon.py:170-179):
    a uint8 HWC image tensor -> normalized float CHW [3, S, S], with the same draws as the
    batched kernels. Each call advances an internal counter, so repeated calls on one image
    give independent views (use with :class:`TwoCropTransform`)."""

    def __init__(self, cfg: AugConfig, seed: int = 0):
        self.cfg = dataclasses.replace(cfg, n_views=1)
        self.seed = int(seed)
        self._calls = 0

    def __call__(self, img: torch.Tensor) -> torch.Tensor:
        assert img.dtype == torch.uint8 and img.dim() == 3 and img.shape[2] == 3, "uint8 HWC image"
        self._calls += 1
        out = augment_reference(img.unsqueeze(0), torch.zeros(1, dtype=torch.long), self.cfg,
                                _mix64((self.seed * 0x9E3779B97F4A7C15 + self._calls) & M64))
        return out[0, :, :, :3].permute(2, 0, 1).contiguous()


class TwoCropTransform:
    """Two independently augmented views of one sample (reference util.py:10-16). The
    training engines draw both views of a whole batch in one GPU launch instead
    (:func:`gpu_augment` with ``n_views=2``); this wrapper serves per-sample pipelines."""

    def __init__(self, transform):
        self.transform = transform

    def __call__(self, x):
        return [self.transform(x), self.transform(x)]
