#!/usr/bin/env python3
"""Time the memory-bound 1x1 dgrads of the bottleneck backward per tile config: plain, and
with the fused epilogue the step runs (residual addend + the next BN's backward statistics
over its input ya and ReLU bits), to see how far each runs from the HBM roofline.

python tools/dgrad_epi_probe.py [--iters 30]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext

# (name, N, H, K (dy channels), C (dx channels)): conv1 of an identity bottleneck, per stage
SHAPES = [("l1c1", 512, 32, 64, 256), ("l2c1", 512, 16, 128, 512), ("l3c1", 512, 8, 256, 1024),
          ("l4c1", 512, 4, 512, 2048)]


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
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--cfgs", default="-1,0,1,2,3,4")
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for name, N, H, K, C in SHAPES:
        dy = torch.randn(N, H, H, K, device=dev).bfloat16()
        wt = (torch.randn(C, 1, 1, K, device=dev) * 0.05).bfloat16()
        add = torch.randn(N, H, H, C, device=dev).bfloat16()
        ya = torch.randn(N, H, H, C, device=dev).bfloat16()
        ma = torch.zeros(C, device=dev)
        bits = torch.randint(0, 255, (N * H * H * C // 8,), device=dev, dtype=torch.uint8)
        out = torch.empty_like(add)
        mb = 2 * N * H * H * (K + C)           # plain: dy read + dx write (bf16)
        me = mb + 2 * N * H * H * C * 2 + N * H * H * C // 8   # + addend + ya + bits
        for cfg in cfgs:
            tp = timeit(lambda: m.conv_dgrad(dy, wt, H, H, 1, 0, cfg, out), a.iters)
            te = timeit(lambda: m.conv_dgrad_bnstat(dy, wt, H, H, 1, 0, cfg, out, add, None, ya, ma,
                                                    mask_bits=bits), a.iters)
            tm = timeit(lambda: m.conv_dgrad_bnstat(dy, wt, H, H, 1, 0, cfg, out, add, None, torch.empty(0, device=dev,
                                                    dtype=torch.bfloat16), ma, mask_bits=bits, store_masked=1),
                        a.iters)
            print(f"{name} cfg {cfg:2d}: plain {tp:7.1f} us {mb / tp / 1e6:5.2f} TB/s | addend+stats {te:7.1f} us "
                  f"{me / te / 1e6:5.2f} TB/s | masked no-ya {tm:7.1f} us", flush=True)
    # 3x3 stride-1 dgrads of the bottleneck's conv2 with the BN1-backward statistics epilogue
    # (ya + ReLU bits, no addend), per stage
    for name, N, H, C in [("l1c2", 512, 32, 64), ("l2c2", 512, 16, 128), ("l3c2", 512, 8, 256)]:
        dy = torch.randn(N, H, H, C, device=dev).bfloat16()
        wt = (torch.randn(C, 3, 3, C, device=dev) * 0.05).bfloat16()
        ya = torch.randn(N, H, H, C, device=dev).bfloat16()
        ma = torch.zeros(C, device=dev)
        bits = torch.randint(0, 255, (N * H * H * C // 8,), device=dev, dtype=torch.uint8)
        out = torch.empty_like(ya)
        for cfg in cfgs:
            tp = timeit(lambda: m.conv_dgrad(dy, wt, H, H, 1, 1, cfg, out), a.iters)
            te = timeit(lambda: m.conv_dgrad_bnstat(dy, wt, H, H, 1, 1, cfg, out, None, None, ya, ma, mask_bits=bits),
                        a.iters)
            print(f"{name} cfg {cfg:2d}: plain {tp:7.1f} us | stats {te:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
