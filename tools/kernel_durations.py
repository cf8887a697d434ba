#!/usr/bin/env python3
"""Per-dispatch device durations from a ``rocprofv3 --kernel-trace`` run, grouped by kernel
(template arguments kept) and grid size: count, median, mean and min in µs.

python tools/kernel_durations.py <dir holding run_kernel_trace.csv> [--match SUBSTR ...]
"""
import argparse
import csv
import os
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", nargs="*", default=[])
    a = ap.parse_args()
    rows = csv.DictReader(open(os.path.join(a.dir, "run_kernel_trace.csv")))
    by = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
        if a.match and not any(m in name for m in a.match):
            continue
        by[(name, r.get("Grid_Size", ""))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':70s} {'grid':>10s} {'n':>6s} {'med_us':>8s} {'mean_us':>8s} {'min_us':>8s}")
    for (name, grid), d in sorted(by.items()):
        print(f"{name:70s} {grid:>10s} {len(d):6d} {statistics.median(d):8.2f} {statistics.fmean(d):8.2f} "
              f"{min(d):8.2f}")


if __name__ == "__main__":
    main()
