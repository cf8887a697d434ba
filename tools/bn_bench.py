#!/usr/bin/env python3
"""Bandwidth of the BatchNorm elementwise kernels on ResNet-50 (CIFAR, 512 views) shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    m = _ext.require()
    dev = torch.device("cuda")
    for (N, H, C) in [(512, 32, 64), (512, 32, 256), (512, 16, 128), (512, 8, 1024), (512, 4, 2048)]:
        y = torch.randn(N, H, H, C, device=dev).bfloat16()
        d = torch.randn_like(y)
        r = torch.randn_like(y)
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        mu, iv = torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5
        nb = y.numel() * 2
        out = m.bn_apply(y, sc, sh, None, None, None, 0, True)
        ca = m.bn_bwd_coef(m.bn_bwd_reduce(d, out, y, mu), float(N * H * H), sc, mu, iv)[0]
        cases = {
            "copy(torch)": (lambda: y.clone(), 2),
            "apply(relu)": (lambda: m.bn_apply(y, sc, sh, None, None, None, 0, True), 2),
            "apply(+res)": (lambda: m.bn_apply(y, sc, sh, r, None, None, 2, True), 3),
            "bwd_reduce(out)": (lambda: m.bn_bwd_reduce(d, out, y, mu), 3),
            "bwd_reduce(mask)": (lambda: m.bn_bwd_reduce(d, None, y, mu, msc=sc, msh=sh), 2),
            "bwd_apply(out)": (lambda: m.bn_bwd_apply(d, out, y, ca), 4),
            "bwd_apply(mask)": (lambda: m.bn_bwd_apply(d, None, y, ca, msc=sc, msh=sh), 3),
        }
        for name, (fn, passes) in cases.items():
            us = timeit(fn)
            print(f"[{N},{H},{H},{C}] {name:18s} {us:8.1f} us  {passes * nb / us / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
