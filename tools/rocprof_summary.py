#!/usr/bin/env python3
"""Summarise a ``rocprofv3 --kernel-trace --stats`` run into per-step kernel time.

Usage: python tools/rocprof_summary.py <rocprof output dir> --steps N [--title ...] [--all]

Default (step window): from the ``*_kernel_trace.csv``, only the kernels
of the LAST N complete training steps -- step boundaries are the starts of ``wprep_kernel``
(the per-step weight conversion, every step's first kernel) -- so set-up work (model init,
data upload, capture or autotune steps, the first-launch copies) never shows up as
per-step cost. ``--all``: the whole run's ``*_kernel_stats.csv`` divided by N (the old
behaviour; mixes set-up kernels into the per-step figures).

Kernels are grouped by family (template arguments kept, long library kernel names
truncated); prints ms/step, calls/step and share of total.
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
    ap.add_argument("--all", action="store_true", help="whole-run kernel stats / steps (includes set-up)")
    a = ap.parse_args()
    tot = defaultdict(float)
    calls = defaultdict(float)
    traces = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if traces and not a.all:
        rows = []
        for f in traces:
            with open(f) as fh:
                rows += list(csv.DictReader(fh))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        starts = [int(r["Start_Timestamp"]) for r in rows if "wprep_kernel" in r["Kernel_Name"]]
        n = int(a.steps)
        if len(starts) < n + 1:
            raise SystemExit(f"{len(starts)} step boundaries (wprep_kernel) in the trace, need {n + 1}")
        t0, t1 = starts[-n - 1], starts[-1]
        for r in rows:
            s = int(r["Start_Timestamp"])
            if t0 <= s < t1:
                k = family(r["Kernel_Name"])
                tot[k] += int(r["End_Timestamp"]) - s
                calls[k] += 1
        scope = f"step window: the last {n} complete steps ({(t1 - t0) / n / 1e6:.3f} ms wall each)"
    else:
        files = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
        if not files:
            raise SystemExit(f"no *kernel_stats.csv under {a.dir}")
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = family(row["Name"])
                    tot[k] += float(row["TotalDurationNs"])
                    calls[k] += float(row["Calls"])
        scope = "whole run / steps (includes set-up kernels)"
    total = sum(tot.values())
    if a.title:
        print(a.title)
    print(f"# {scope}")
    print(f"TOTAL kernel time per step: {total / a.steps / 1e6:.3f} ms")
    for k in sorted(tot, key=tot.get, reverse=True)[: a.top]:
        print(f"{tot[k] / a.steps / 1e6:8.3f} ms/step {calls[k] / a.steps:8.1f} calls/step "
              f"{100 * tot[k] / total:6.1f}%  {k}")


if __name__ == "__main__":
    main()
