"""Time one wgrad GEMM over tile configs x explicit split counts (grid-fill study).
Usage: python tools/wgrad_split_probe.py N,H,W,C,K,R,stride,pad cfgs splits"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext
from tools.conv_bench import timeit

N, H, W, C, K, R, st, pad = [int(v) for v in sys.argv[1].split(",")]
cfgs = [int(c) for c in sys.argv[2].split(",")]
splits = [int(s) for s in sys.argv[3].split(",")]
m = _ext.require()
dev = torch.device("cuda")
x = torch.randn(N, H, W, C, device=dev).bfloat16()
P = (H + 2 * pad - R) // st + 1
dy = torch.randn(N, P, P, K, device=dev).bfloat16()
out = torch.empty(K, R, R, C, device=dev, dtype=torch.float32)
print(f"auto {timeit(lambda: m.conv_wgrad(dy, x, R, R, st, pad, 0, -1, out), 20):.1f} us")
for c in cfgs:
    row = [f"{s}:{timeit(lambda: m.conv_wgrad(dy, x, R, R, st, pad, s, c, out), 20):.1f}" for s in splits]
    print(f"cfg{c} " + " ".join(row), flush=True)
