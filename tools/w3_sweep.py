#!/usr/bin/env python3
"""Split-count sweep of the dedicated wgrad kernels against the generic implicit-GEMM wgrad
(cfg -2) on the CIFAR ResNet-50 shapes at 512 views: the tap-reuse 3x3 kernel (cfg 9,
csrc/kernels/wgrad3x3.hip) and the stride-1 1x1 kernel (cfg 10, csrc/kernels/wgrad1x1.hip).

python tools/w3_sweep.py [--iters 20] [--kind 3x3|1x1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext

SHAPES = [("l1.c2", 512, 32, 64, 64), ("l2.c2", 512, 16, 128, 128), ("l3.c2", 512, 8, 256, 256),
          ("l4.c2", 512, 4, 512, 512)]
# (name, N, H, C_in, K_out) of the stride-1 1x1 convs the 1x1 kernel takes
SHAPES_1X1 = [("l2.0.c1", 512, 32, 256, 128), ("l2.x.c1", 512, 16, 512, 128), ("l2.x.c3", 512, 16, 128, 512),
              ("l3.0.c1", 512, 16, 512, 256), ("l3.x.c1", 512, 8, 1024, 256), ("l3.x.c3", 512, 8, 256, 1024),
              ("l4.0.c1", 512, 8, 1024, 512), ("l4.x.c1", 512, 4, 2048, 512), ("l4.x.c3", 512, 4, 512, 2048)]


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
    ap.add_argument("--kind", default="3x3", choices=["3x3", "1x1"])
    a = ap.parse_args()
    R, pad, cfg, bm, bn = (3, 1, 9, 64, 64) if a.kind == "3x3" else (1, 0, 10, 128, 256)
    m = _ext.require()
    dev = torch.device("cuda")
    for name, N, H, C, K in (SHAPES if a.kind == "3x3" else SHAPES_1X1):
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        dy = torch.randn(N, H, H, K, device=dev).bfloat16()
        sink = torch.zeros(K, R, R, C, device=dev)
        steps = N * H * H // 32
        tiles = (K // bm) * (C // (bn if C % bn == 0 else 128))
        gen = timed(lambda: m.conv_wgrad(dy, x, R, R, 1, pad, 0, -2, sink, True), a.iters)
        row = [f"{name:6s} tiles={tiles:3d} steps={steps:6d} generic={gen:6.1f}"]
        for sp in (2, 4, 8, 16, 32, 64, 128, 192, 256, 384, 512):
            if sp * tiles < 64 or sp * tiles > 1024 or steps // sp < 8:
                continue
            t = timed(lambda: m.conv_wgrad(dy, x, R, R, 1, pad, sp, cfg, sink, True), a.iters)
            row.append(f"{sp}:{t:.1f}")
        print(" ".join(row), flush=True)


if __name__ == "__main__":
    main()
