#!/usr/bin/env python3
"""Main-loop timeline of one conv launch (SDX_IGEMM_TRACE=1 is set here): block 0, waves 0
(group 0) and 4 (group 1) of the ping-pong loop; per K-tile the cycles of the load segment
(fragment reads + DMA issue + wait), the barrier wait, and the MFMA issue.

python tools/igemm_trace.py --mode fwd --shape 512,8,8,256,256,3,1,1 --cfg 6
"""
import argparse
import os
import sys

os.environ["SDX_IGEMM_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from simclr_pytorch_distributed_amd.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fwd", choices=["fwd", "dgrad"])
    ap.add_argument("--shape", default="512,8,8,256,256,3,1,1")
    ap.add_argument("--cfg", type=int, default=6)
    a = ap.parse_args()
    N, H, W, C, K, R, st, pad = [int(v) for v in a.shape.split(",")]
    m = _ext.require()
    dev = torch.device("cuda")
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
    P = (H + 2 * pad - R) // st + 1
    dy = torch.randn(N, P, P, K, device=dev).bfloat16()
    wt = w.permute(3, 1, 2, 0).contiguous()
    fn = {"fwd": lambda: m.conv_fwd(x, w, st, pad, True, a.cfg),
          "dgrad": lambda: m.conv_dgrad(dy, wt, H, W, st, pad, a.cfg)}[a.mode]
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = m.igemm_trace().tolist()
    S = len(t[0])
    for g in range(2):
        r = t[g]
        t0 = r[0]
        rt = (r[S - 1] - r[S - 5]) / 100e6      # seconds (100 MHz realtime)
        cyc = r[S - 2] - t0
        print(f"wave {4 * g}: total {cyc} cycles, {rt * 1e6:.2f} us -> {cyc / rt / 1e9 if rt else 0:.2f} GHz; "
              f"prologue {r[1] - t0}, loop {r[S - 4] - r[1]}, epilogue {r[S - 2] - r[S - 4]} "
              f"(staged at +{r[S - 3] - r[S - 4]})")
        if r[4] == 0 and r[2] > 0:
            # DEPTH 6 stamps only E2 (first-half MFMAs issued) and E3 (after the barrier)
            rows = []
            kt = 0
            while 2 + 3 * (kt + 1) < S - 5 and r[2 + 3 * (kt + 1)] > 0 and kt < 159:
                rows.append((r[3 + 3 * kt] - r[2 + 3 * kt], r[2 + 3 * (kt + 1)] - r[3 + 3 * kt]))
                kt += 1
            if rows:
                n = len(rows)
                print(f"  {n} K-tiles: vmcnt+barrier wait {sum(x[0] for x in rows) / n:.0f}  "
                      f"half2 + next half1 {sum(x[1] for x in rows) / n:.0f} cycles (mean)")
                for x in rows[:4] + rows[-3:]:
                    print("   ", x)
            continue
        rows = []
        kt = 0
        while 4 + 3 * kt < S - 5 and r[4 + 3 * kt] > 0 and kt < 160:
            a0 = r[1] if kt == 0 else r[4 + 3 * (kt - 1)]
            rows.append((r[2 + 3 * kt] - a0, r[3 + 3 * kt] - r[2 + 3 * kt], r[4 + 3 * kt] - r[3 + 3 * kt]))
            kt += 1
        if rows:
            n = len(rows)
            avg = [sum(x[i] for x in rows) / n for i in range(3)]
            print(f"  {n} K-tiles: load seg {avg[0]:.0f}  barrier wait {avg[1]:.0f}  mfma issue {avg[2]:.0f} cycles (mean)")
            for i, x in enumerate(rows[:6] + rows[-3:]):
                print("   ", x)


if __name__ == "__main__":
    main()
