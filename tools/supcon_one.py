#!/usr/bin/env python3
"""Fused NT-Xent/SupCon loss kernels alone (forward + backward) for timing and rocprofv3
counter collection: N anchors x N contrast rows of dim 128 (N = 2 x batch).

python tools/supcon_one.py --n 512 --iters 20
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from simclr_pytorch_distributed_amd.losses.supcon import DistributedContrastiveLoss
    crit = DistributedContrastiveLoss("SimCLR", 0.5, backend="native")
    f = torch.randn(a.n, a.dim, device="cuda", requires_grad=True)

    def step():
        loss = crit(f)
        loss.backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        step()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / a.iters * 1e3
    flops = 2 * 2 * a.n * a.n * a.dim * 3   # fwd logits + bwd (dA, dC) GEMMs, bf16x3 split precision
    print(f"supcon fwd+bwd n={a.n} d={a.dim}: {us:.1f} us ({flops / us / 1e6:.1f} TFLOP/s incl. 3-pass split)")


if __name__ == "__main__":
    main()
