#!/usr/bin/env python3
"""Split-count sweep of the tap-reuse 3x3 wgrad (cfg 9, csrc/kernels/wgrad3x3.hip) on the
CIFAR ResNet-50 3x3 shapes at 512 views, against the generic implicit-GEMM wgrad (auto).

python tools/w3_sweep.py [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext

SHAPES = [("l1.c2", 512, 32, 64, 64), ("l2.c2", 512, 16, 128, 128), ("l3.c2", 512, 8, 256, 256),
          ("l4.c2", 512, 4, 512, 512)]


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    for name, N, H, C, K in SHAPES:
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dy = torch.randn(N, H, H, K, device=dev).bfloat16()
        sink = torch.zeros(K, 3, 3, C, device=dev)
        steps = N * H * H // 32
        tiles = (K // 64) * (C // 64)
        gen = timed(lambda: m.conv_wgrad(dy, x, 3, 3, 1, 1, 0, -2, sink, True), a.iters)
        row = [f"{name:6s} tiles={tiles:3d} steps={steps:6d} generic={gen:6.1f}"]
        for sp in (2, 4, 8, 16, 32, 64, 128, 192, 256, 384, 512):
            if sp * tiles < 64 or sp * tiles > 2048 or steps // sp < 8:
                continue
            t = timed(lambda: m.conv_wgrad(dy, x, 3, 3, 1, 1, sp, 9, sink, True),
                      a.iters)
            row.append(f"{sp}:{t:.1f}")
        print(" ".join(row), flush=True)


if __name__ == "__main__":
    main()
