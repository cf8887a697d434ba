#!/usr/bin/env python3
"""Per-kernel HBM traffic of the training step from two rocprofv3 counter passes (FETCH_SIZE,
WRITE_SIZE; they do not fit one pass) joined with the kernel-trace summary of an ordinary
run: MB moved per step and the effective TB/s at the in-step kernel time.

python tools/hbm_traffic.py <fetch dir> <write dir> <summary.txt from tools/rocprof_summary.py>
Steps are counted by sgd_kernel dispatches (one per step).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    tot, steps = defaultdict(float), 0
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name)[:70]
        if r.get("Counter_Name", counter) != counter:
            continue
        tot[name] += float(r["Counter_Value"])
        if name.startswith("sgd_kernel"):
            steps += 1
    return tot, max(steps, 1)


def main():
    fetch, sf = load(sys.argv[1], "FETCH_SIZE")
    write, sw = load(sys.argv[2], "WRITE_SIZE")
    ms = {}
    for line in open(sys.argv[3]):
        m = re.match(r"\s*([0-9.]+) ms/step\s+([0-9.]+) calls/step\s+[0-9.]+%\s+(.*)", line)
        if m:
            ms[m.group(3).replace("void ", "")[:70]] = float(m.group(1))
    rows = []
    for k in set(fetch) | set(write):
        rd, wr = fetch.get(k, 0.0) / sf / 1e3, write.get(k, 0.0) / sw / 1e3     # KB -> MB per step
        t = next((v for n, v in ms.items() if n.startswith(k[:60])), None)
        rows.append((rd + wr, k, rd, wr, t))
    tot_rd = sum(r[2] for r in rows)
    tot_wr = sum(r[3] for r in rows)
    print(f"# HBM traffic per step: read {tot_rd:.0f} MB, write {tot_wr:.0f} MB ({sf} steps counted)")
    print(f"{'MB/step':>9} {'read':>8} {'write':>8} {'ms/step':>8} {'TB/s':>6}  kernel")
    for tot, k, rd, wr, t in sorted(rows, reverse=True)[:40]:
        bw = f"{tot / t / 1e3:6.2f}" if t else "     -"
        print(f"{tot:9.1f} {rd:8.1f} {wr:8.1f} {t if t else 0:8.3f} {bw}  {k}")


if __name__ == "__main__":
    main()
