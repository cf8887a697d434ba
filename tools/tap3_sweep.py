#!/usr/bin/env python3
"""Per-shape timing of every 3x3 stride-1 conv of the CIFAR ResNet-50 (512 views) across the
implicit-GEMM tile configs and the tap-reuse configs (11-13), fwd and dgrad, in one process
(interleaved rounds, median): python tools/tap3_sweep.py [--iters 30] [--rounds 3]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from simclr_pytorch_distributed_amd.ops import _ext  # noqa: E402

SHAPES = [("l1", 512, 32, 64, 64), ("l2", 512, 16, 128, 128), ("l3", 512, 8, 256, 256), ("l4", 512, 4, 512, 512)]
CFGS = [1, 4, 6, 11, 12, 13]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, N, H, C, K in SHAPES:
        x = torch.randn(N, H, H, C, device=dev).bfloat16()
        w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).bfloat16()
        dy = torch.randn(N, H, H, K, device=dev).bfloat16()
        wt = w.permute(3, 1, 2, 0).contiguous()
        fl = 2.0 * N * H * H * K * 9 * C
        for mode in ("fwd", "dgrad"):
            res = {}
            for _ in range(a.rounds):
                for cfg in [-1] + CFGS:
                    fn = (lambda c=cfg: m.conv_fwd(x, w, 1, 1, True, c)) if mode == "fwd" else \
                        (lambda c=cfg: m.conv_dgrad(dy, wt, H, H, 1, 1, c))
                    try:
                        fn()
                    except RuntimeError:
                        continue
                    torch.cuda.synchronize()
                    st.record()
                    for _ in range(a.iters):
                        fn()
                    en.record()
                    torch.cuda.synchronize()
                    res.setdefault(cfg, []).append(st.elapsed_time(en) / a.iters * 1e3)
            line = " ".join(f"cfg{c if c >= 0 else 'auto'} {statistics.median(v):6.1f}us/{fl / statistics.median(v) / 1e6:5.0f}TF"
                            for c, v in res.items())
            print(f"{name} {mode:5s} {line}", flush=True)


if __name__ == "__main__":
    main()
