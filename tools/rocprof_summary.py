#!/usr/bin/env python3
"""Summarise a ``rocprofv3 --kernel-trace --stats`` run into per-step kernel time.

Usage: python tools/rocprof_summary.py <rocprof output dir> --steps N [--title ...]

Reads every ``*_kernel_stats.csv`` under the directory (columns Name, Calls,
TotalDurationNs, ...), groups kernels by family (template arguments kept, long library
kernel names truncated) and prints ms/step, calls/step and share of total.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
from collections import defaultdict


def family(name: str) -> str:
    name = name.strip()
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    # drop the argument list, keep template args
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    return name[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=float, required=True)
    ap.add_argument("--title", default="")
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_stats.csv under {a.dir}")
    tot = defaultdict(float)
    calls = defaultdict(float)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = family(row["Name"])
                tot[k] += float(row["TotalDurationNs"])
                calls[k] += float(row["Calls"])
    total = sum(tot.values())
    if a.title:
        print(a.title)
    print(f"TOTAL kernel time per step: {total / a.steps / 1e6:.3f} ms")
    for k in sorted(tot, key=tot.get, reverse=True)[: a.top]:
        print(f"{tot[k] / a.steps / 1e6:8.3f} ms/step {calls[k] / a.steps:8.1f} calls/step "
              f"{100 * tot[k] / total:6.1f}%  {k}")


if __name__ == "__main__":
    main()
