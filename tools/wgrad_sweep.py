"""WGRAD tile/split sweep on the ResNet-50 CIFAR shapes (512 views per GPU).

For every distinct weight-gradient GEMM, times the native split-K wgrad (kernel + slab
reduce) for each tile config and a range of split counts, and prints the auto choice's
time next to the best found. Used to calibrate ``conv_wgrad``'s split / tile heuristic
(csrc/bindings/conv_bn_ops.cpp).

Usage: python tools/wgrad_sweep.py [--views 512] [--iters 20] [--cfgs 0,1,2,3,4]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext
from tools.conv_bench import resnet50_convs, timeit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfgs", default="0,1,2,3,4")
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    cfgs = [int(c) for c in a.cfgs.split(",")]
    tot_auto = tot_best = 0.0
    print(f"{'shape':10s} {'M':>5s} {'N':>5s} {'Kd':>7s} {'auto_us':>8s} {'best_us':>8s} best(cfg,splits)  top3",
          flush=True)
    for (name, N, H, W, C, K, R, st, pad, cnt) in resnet50_convs(a.views):
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, K, device=dev).bfloat16()
        Kd = N * P * P
        out = torch.empty(K, R, R, C, device=dev, dtype=torch.float32)
        ref = m.conv_wgrad(dy, x, R, R, st, pad, 0, -1).clone()
        t_auto = timeit(lambda: m.conv_wgrad(dy, x, R, R, st, pad, 0, -1, out), a.iters)
        res = []
        for cfg in cfgs:
            for sp in (1, 2, 4, 8, 16, 32, 64, 128, 256):
                if Kd // sp < 256:
                    continue
                got = m.conv_wgrad(dy, x, R, R, st, pad, sp, cfg, out)
                err = (got - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                if err > 1e-3:
                    print(f"  MISMATCH {name} cfg={cfg} splits={sp} rel={err:.2e}", flush=True)
                    continue
                res.append((timeit(lambda: m.conv_wgrad(dy, x, R, R, st, pad, sp, cfg, out), a.iters), cfg, sp))
        res.sort()
        tb, cb, sb = res[0]
        tot_auto += t_auto * cnt
        tot_best += tb * cnt
        top = " ".join(f"{t:.1f}@{c},{s}" for t, c, s in res[:3])
        print(f"{name:10s} {K:5d} {R * R * C:5d} {Kd:7d} {t_auto:8.1f} {tb:8.1f} ({cb},{sb})  {top}  x{cnt}",
              flush=True)
    print(f"TOTAL wgrad auto {tot_auto / 1e3:.3f} ms  best {tot_best / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
