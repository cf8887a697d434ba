"""Cost of the fused BN-backward statistics epilogue: conv_dgrad vs conv_dgrad_bnstat (ReLU
mask from a bitmask, the block-internal BN case) on every ResNet-50 dgrad shape.

Usage: python tools/bst_ab.py [--views 512] [--iters 20]
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
    ap.add_argument("--cfgs", default="-1", help="comma-separated tile configs to time the bnstat variant with")
    ap.add_argument("--only", default="", help="comma-separated shape names")
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    tp = tb = 0.0
    print(f"{'shape':10s} {'plain_us':>9s} {'bnstat_us':>10s} {'extra_us':>9s}")
    for (name, N, H, W, C, K, R, st, pad, cnt) in resnet50_convs(a.views):
        if name == "stem" or (a.only and name not in a.only.split(",")):
            continue
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, K, device=dev).bfloat16()
        wt = (torch.randn(C, R, R, K, device=dev) * 0.05).bfloat16()
        y = torch.randn(N, H, W, C, device=dev).bfloat16()
        mu = torch.zeros(C, device=dev)
        bits = torch.randint(0, 256, (y.numel() // 8,), dtype=torch.uint8, device=dev)
        t0 = timeit(lambda: m.conv_dgrad(dy, wt, H, W, st, pad, -1), a.iters)
        ts = [timeit(lambda: m.conv_dgrad_bnstat(dy, wt, H, W, st, pad, int(cf), ya=y, ma=mu, mask_bits=bits), a.iters)
              for cf in a.cfgs.split(",")]
        t1 = ts[0]
        tp += t0 * cnt
        tb += t1 * cnt
        alt = "  " + " ".join(f"cfg{cf}:{t:.1f}" for cf, t in zip(a.cfgs.split(",")[1:], ts[1:])) if len(ts) > 1 else ""
        print(f"{name:10s} {t0:9.1f} {t1:10.1f} {t1 - t0:9.1f}  x{cnt}{alt}", flush=True)
    print(f"TOTAL plain {tp / 1e3:.3f} ms  bnstat {tb / 1e3:.3f} ms  extra {(tb - tp) / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
