#!/usr/bin/env python3
"""Re-calibration of the fwd / dgrad tile selection: every distinct conv of the CIFAR ResNet-50
(512 views) timed with auto (-1) and every tile config 0-6 (+ the tap-reuse 11-13 where they
apply), in one process, interleaved rounds, median. Prints per shape the auto time, the best
config and its time, and the totals (weighted by the per-step count).

python tools/cfg_sweep.py [--rounds 3] [--iters 20] [--stats 1]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from conv_bench import resnet50_convs  # noqa: E402
from simclr_pytorch_distributed_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    st_ev, en_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cfgs = [-1, 0, 1, 2, 3, 4, 5, 6, 11, 12, 13]
    tot_auto = tot_best = 0.0
    for (name, N, H, W, C, K, R, st, pad, cnt) in resnet50_convs(a.views):
        if name == "stem":
            continue
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, K, device=dev).bfloat16()
        wt = w.permute(3, 1, 2, 0).contiguous()
        ya = torch.randn(N, H, W, C, device=dev).bfloat16()
        mu = torch.zeros(C, device=dev)
        for mode in ("fwd", "dgrad"):
            res = {}
            for _ in range(a.rounds):
                for cfg in cfgs:
                    if mode == "fwd":
                        fn = (lambda c=cfg: m.conv_fwd(x, w, st, pad, True, c))
                    else:   # the step's dgrads carry the BN-backward statistics epilogue
                        fn = (lambda c=cfg: m.conv_dgrad_bnstat(dy, wt, H, W, st, pad, c, None, None, None, ya, mu,
                                                                None, None, None, None, None))
                    try:
                        fn()
                    except RuntimeError:
                        continue
                    torch.cuda.synchronize()
                    st_ev.record()
                    for _ in range(a.iters):
                        fn()
                    en_ev.record()
                    torch.cuda.synchronize()
                    res.setdefault(cfg, []).append(st_ev.elapsed_time(en_ev) / a.iters * 1e3)
            med = {c: statistics.median(v) for c, v in res.items()}
            best = min((c for c in med if c >= 0), key=lambda c: med[c])
            tot_auto += med[-1] * cnt
            tot_best += med[best] * cnt
            flag = "  <-- auto off by %.1f us" % (med[-1] - med[best]) if med[-1] > 1.03 * med[best] else ""
            print(f"{name:10s} {mode:5s} M={N * P * P if mode == 'fwd' else N * H * W:7d} N={K if mode == 'fwd' else C:5d} "
                  f"K={R * R * (C if mode == 'fwd' else K):5d}  auto {med[-1]:7.1f}  best cfg {best:2d} {med[best]:7.1f}  x{cnt}"
                  + "  [" + " ".join(f"{c}:{med[c]:.0f}" for c in sorted(med) if c >= 0) + "]" + flag, flush=True)
    print(f"TOTAL auto {tot_auto / 1e3:.3f} ms, best-per-shape {tot_best / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
