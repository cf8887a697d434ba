"""1x1 wgrad A/B: the 256-row LDS-DMA kernel (wgrad1x1_big_kernel) vs the 128-row
register-ring kernel on the CIFAR ResNet-50 layer 2-4 shapes at 512 views: auto split (the
in-step 128-block target) and a split sweep. Usage: python tools/w1_big_ab.py [--sweep]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext
from tools.conv_bench import timeit

SHAPES = [  # name, N, H, C (x channels), K (dy channels), stride
    ("l2.0.c3", 512, 16, 128, 512, 1), ("l2.0.sc", 512, 32, 256, 512, 2), ("l3.0.c1", 512, 16, 512, 256, 1),
    ("l3.x.c1", 512, 8, 1024, 256, 1), ("l3.x.c3", 512, 8, 256, 1024, 1), ("l3.0.sc", 512, 16, 512, 1024, 2),
    ("l4.0.c1", 512, 8, 1024, 512, 1), ("l4.x.c1", 512, 4, 2048, 512, 1), ("l4.x.c3", 512, 4, 512, 2048, 1),
    ("l4.0.sc", 512, 8, 1024, 2048, 2),
]
m = _ext.require()
dev = torch.device("cuda")
sweep = "--sweep" in sys.argv
tot = [0.0, 0.0]
for name, N, H, C, K, st in SHAPES:
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    P = H // st
    dy = torch.randn(N, P, P, K, device=dev).bfloat16()
    out = torch.empty(K, 1, 1, C, device=dev, dtype=torch.float32)
    row = []
    for big in (0, 1):
        m.wgrad1x1_big_set(2 * big)
        t = timeit(lambda: m.conv_wgrad(dy, x, 1, 1, st, 0, 0, -1, out), 20)
        tot[big] += t
        row.append(t)
    fl = 2.0 * N * P * P * C * K
    line = f"{name:8s} old {row[0]:7.1f} us  big {row[1]:7.1f} us  ({fl / row[1] / 1e6:6.1f} TF/s)"
    if sweep:
        m.wgrad1x1_big_set(2)
        line += "  splits " + " ".join(
            f"{s}:{timeit(lambda: m.conv_wgrad(dy, x, 1, 1, st, 0, s, 10, out), 20):.1f}" for s in (2, 4, 8, 16, 32, 64))
    print(line, flush=True)
m.wgrad1x1_big_set(1)
print(f"TOTAL (one each) old {tot[0]:.1f} us  big {tot[1]:.1f} us")
