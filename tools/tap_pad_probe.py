#!/usr/bin/env python3
"""Per-config timing of the 224x224 config's stride-1 3x3 convs (56x56x64, 28x28x128 at 1024
views): forward with statistics and dgrad, every tile config that accepts the shape —
the padded-row tap tiles (11-13) against the implicit-GEMM tiles (0, 1, 4).

python tools/tap_pad_probe.py [--n 1024] [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext


def timeit(fn, iters):
    for _ in range(2):
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
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    for H, C in [(56, 64), (28, 128)]:
        N, K = a.n, C
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).bfloat16()
        wt = w.permute(3, 1, 2, 0).contiguous()   # [C][R][S][K]
        dy = torch.randn(N, H, H, K, device=dev).bfloat16()
        flops = 2.0 * N * H * H * K * 9 * C
        for cfg in (-1, 0, 1, 4, 11, 12, 13):
            row = f"{H}x{H}x{C} cfg {cfg:3d}:"
            try:
                t = timeit(lambda: m.conv_fwd(x, w, 1, 1, True, cfg), a.iters)
                row += f" fwd+stats {t:8.1f} us {flops / t / 1e6:6.0f} TF/s |"
            except RuntimeError:
                row += " fwd        n/a               |"
            try:
                t = timeit(lambda: m.conv_dgrad(dy, wt, H, H, 1, 1, cfg), a.iters)
                row += f" dgrad {t:8.1f} us {flops / t / 1e6:6.0f} TF/s"
            except RuntimeError:
                row += " dgrad      n/a"
            print(row, flush=True)


if __name__ == "__main__":
    main()
