#!/usr/bin/env python3
"""The BN3 fold's G = dzᵀ·a2 at layer 1 (dz 256 channels, a2 64) as computed today (a
[256][64] output: the generic 256x64 wgrad tile) against its transpose a2ᵀ·dz (a [64][256]
output the dedicated 1x1 wgrad kernels take), stand-alone, 512 views of 32x32.

python tools/gt_probe.py [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    for name, N, H, C3, K3 in [("l1", 512, 32, 256, 64), ("l2", 512, 16, 512, 128)]:
        dz = torch.randn(N, H, H, C3, device=dev).bfloat16()
        a2 = torch.randn(N, H, H, K3, device=dev).bfloat16()
        g = torch.empty(C3, 1, 1, K3, device=dev)
        gt = torch.empty(K3, 1, 1, C3, device=dev)
        t_g = timeit(lambda: m.conv_wgrad(dz, a2, 1, 1, 1, 0, 0, -1, g, False), a.iters)
        t_gt = timeit(lambda: m.conv_wgrad(a2, dz, 1, 1, 1, 0, 0, -1, gt, False), a.iters)
        err = (g.view(C3, K3) - gt.view(K3, C3).t()).abs().max().item() / g.abs().max().item()
        mb = 2 * N * H * H * (C3 + K3) / 1e6
        print(f"{name}: G [{C3}][{K3}] {t_g:7.1f} us ({mb / t_g:.2f} TB/s) | G^T [{K3}][{C3}] {t_gt:7.1f} us "
              f"({mb / t_gt:.2f} TB/s) | rel diff {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
