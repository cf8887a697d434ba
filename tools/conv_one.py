#!/usr/bin/env python3
"""Run ONE native conv pass repeatedly (for rocprofv3 counter collection / A-B timing).

python tools/conv_one.py --mode fwd --shape N,H,W,C,K,R,stride,pad [--cfg -1] [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--shape", default="512,8,8,256,256,3,1,1")
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--nostats", action="store_true")
    a = ap.parse_args()
    N, H, W, C, K, R, st, pad = [int(v) for v in a.shape.split(",")]
    m = _ext.require()
    dev = torch.device("cuda")
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
    P = (H + 2 * pad - R) // st + 1
    dy = torch.randn(N, P, P, K, device=dev).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()
    fn = {"fwd": lambda: m.conv_fwd(x, w, st, pad, not a.nostats, a.cfg),
          "dgrad": lambda: m.conv_dgrad(dy, wt, H, W, st, pad, a.cfg),
          "wgrad": lambda: m.conv_wgrad(dy, x, R, R, st, pad, 0, a.cfg)}[a.mode]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / a.iters * 1e3
    flops = 2.0 * N * P * P * K * R * R * C
    print(f"{a.mode} {a.shape} cfg {a.cfg}: {us:.1f} us  {flops / us / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
