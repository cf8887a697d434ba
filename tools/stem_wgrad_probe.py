#!/usr/bin/env python3
"""Stand-alone sweep of the CIFAR stem's weight gradient (3x3, 3 -> 64 channels with the
input padded to 8, 512 views of 32x32): the last kernel chain of the backward, on the
compute stream. Tile config x split count, including the fp32 split-K reduction.

python tools/stem_wgrad_probe.py [--iters 20]
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
    N, H, Cp, K = 512, 32, 8, 64
    x = torch.randn(N, H, H, Cp, device=dev).bfloat16()
    dy = torch.randn(N, H, H, K, device=dev).bfloat16()
    ref = m.conv_wgrad(dy, x, 3, 3, 1, 1, 0, -1)
    print(f"auto: {timeit(lambda: m.conv_wgrad(dy, x, 3, 3, 1, 1, 0, -1), a.iters):7.1f} us", flush=True)
    for cfg in (0, 1, 2, 3):
        for splits in (32, 64, 128, 256, 512):
            try:
                t = timeit(lambda: m.conv_wgrad(dy, x, 3, 3, 1, 1, splits, cfg), a.iters)
                out = m.conv_wgrad(dy, x, 3, 3, 1, 1, splits, cfg)
                err = ((out - ref).abs().max() / ref.abs().max()).item()
                print(f"cfg {cfg} splits {splits:4d}: {t:7.1f} us (rel diff {err:.1e})", flush=True)
            except RuntimeError as e:
                print(f"cfg {cfg} splits {splits:4d}: n/a ({str(e)[:60]})", flush=True)


if __name__ == "__main__":
    main()
