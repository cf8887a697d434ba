#!/usr/bin/env python3
"""Per-kernel cost under hipGraph replay vs eager launches (the graphed
step's kernels each ran 1.3-2x their eager time).

For a few representative kernels of the step -- a compute-bound conv (l3 3x3 fwd), a
memory-bound elementwise pass (torch add over 64 MB), a small latency-bound launch (torch
add over 64 KB) -- time N back-to-back eager launches against one replay of a graph that
captured the same N launches, on the same buffers.

python tools/graph_probe.py [--n 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50)
    a = ap.parse_args()
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    dev = torch.device("cuda")
    n = a.n
    x3 = torch.randn(512, 8, 8, 256, device=dev).bfloat16()
    w3 = (torch.randn(256, 3, 3, 256, device=dev) * 0.05).bfloat16()
    big = torch.randn(16 << 20, device=dev)
    small = torch.randn(16 << 10, device=dev)
    ops = {
        "conv_l3_3x3_fwd": lambda: m.conv_fwd(x3, w3, 1, 1, True, -1),
        "add_64MB": lambda: big.add(1.0),
        "add_64KB": lambda: small.add(1.0),
    }
    for name, op in ops.items():
        def eager():
            for _ in range(n):
                op()
        te = timed(eager)
        for side in (False, True):
            s = torch.cuda.Stream(priority=-1) if side else torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(3):
                    op()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s if side else None):
                for _ in range(n):
                    op()
            tg = timed(g.replay)
            print(f"{name:18s} eager {te / n:8.2f} us/launch   graph{'(prio stream)' if side else ''} "
                  f"{tg / n:8.2f} us/launch   ratio {tg / te:.2f}", flush=True)
            del g


if __name__ == "__main__":
    main()
