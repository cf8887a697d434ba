#!/usr/bin/env python3
"""1x1 stride-1 weight gradients (plain GEMMs dW[co][ci] = Σ_pix dy[pix][co]·x[pix][ci]):
native igemm WGRAD vs hipBLASLt through torch.mm (bf16 out, and fp32 out via mm.dtype).

python tools/wgrad_vs_blas.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.ops import _ext

SHAPES = [  # (pixels, cout, cin) of the ResNet-50 CIFAR 1x1 convs at 512 images
    ("l1.c1", 524288, 64, 256), ("l1.c3", 524288, 256, 64), ("l1.sc", 524288, 256, 64),
    ("l2.c1", 131072, 128, 512), ("l2.c3", 131072, 512, 128),
    ("l3.c1", 32768, 256, 1024), ("l3.c3", 32768, 1024, 256),
    ("l4.c1", 8192, 512, 2048), ("l4.c3", 8192, 2048, 512),
]


def bench(fn, iters=20):
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
    m = _ext.require()
    dev = torch.device("cuda")
    print(f"{'shape':8s} {'P':>7s} {'co':>5s} {'ci':>5s} {'native_us':>10s} {'mm_bf16_us':>10s} {'mm_f32out_us':>12s} {'TF/s nat':>8s} {'TF/s f32':>8s}")
    for name, P, co, ci in SHAPES:
        side = int(P ** 0.5)
        N = P // (side * side) if P % (side * side) == 0 else 1
        dy = torch.randn(P, co, device=dev).bfloat16()
        x = torch.randn(P, ci, device=dev).bfloat16()
        dy4 = dy.view(1, 1, P, co)
        x4 = x.view(1, 1, P, ci)
        nat = bench(lambda: m.conv_wgrad(dy4, x4, 1, 1, 1, 0, 0, -1))
        mmb = bench(lambda: torch.mm(dy.t(), x))
        try:
            mmf = bench(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        except Exception:  # noqa: BLE001
            mmf = float("nan")
        ref = torch.mm(dy.t().float(), x.float())
        got = m.conv_wgrad(dy4, x4, 1, 1, 1, 0, 0, -1).view(co, ci)
        err = ((got - ref).norm() / ref.norm()).item()
        fl = 2.0 * P * co * ci
        print(f"{name:8s} {P:7d} {co:5d} {ci:5d} {nat:10.1f} {mmb:10.1f} {mmf:12.1f} {fl / nat / 1e6:8.1f} {fl / mmf / 1e6:8.1f}  err={err:.1e}")


if __name__ == "__main__":
    main()
