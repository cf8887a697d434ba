#!/usr/bin/env python3
"""From a rocprofv3 kernel trace of bench.py: wall time of the last training step
(wprep_kernel start to wprep_kernel start: the per-step weight conversion is the step's first
kernel; the optimizer update runs per gradient bucket), GPU-busy time (union of kernel intervals over all
streams) and idle gaps, plus the busiest kernels of that step.

python tools/step_timeline.py <rocprof dir> [--dump FILE]
  --dump: every kernel of that step (start / end in us from the step start, stream or
  queue id, grid, name) for offline analysis
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        r["Kernel_Name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "wprep_kernel" in r["Kernel_Name"]]
    a, b = idx[-2] - 1, idx[-1] - 1
    t0, t1 = int(rows[a + 1]["Start_Timestamp"]), int(rows[b + 1]["Start_Timestamp"])
    busy, cur, gaps = 0, t0, []
    per = defaultdict(float)
    prev_name = rows[a]["Kernel_Name"]
    where = []
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        per[r["Kernel_Name"].split("(")[0][:80]] += (e - s) / 1e3
        if s > cur:
            gaps.append((s - cur) / 1e3)
            where.append(((s - cur) / 1e3, (cur - t0) / 1e3, prev_name[:60], r["Kernel_Name"][:60]))
        if e > cur:
            prev_name = r["Kernel_Name"]
        if e <= cur:
            continue
        busy += e - max(s, cur)
        cur = e
    print(f"last step: wall {(t1 - t0) / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us "
          f"in {len(gaps)} gaps (largest {max(gaps) if gaps else 0:.1f} us), kernels {b - a}")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  {v:8.1f} us  {k}")
    print("largest gaps (us, at us into the step, after -> before):")
    for g, at, pn, nn in sorted(where, reverse=True)[:15]:
        print(f"  {g:7.1f} @{at:8.1f}  {pn.split('(')[0]}  ->  {nn.split('(')[0]}")
    # per-stream busy time in the step (union per stream) and their overlap
    key = next((k for k in ("Stream_Id", "Queue_Id", "Stream_ID", "Queue_ID") if k in rows[0]), None)
    if "--dump" in sys.argv:
        with open(sys.argv[sys.argv.index("--dump") + 1], "w") as fo:
            for r in rows[a + 1:b + 1]:
                fo.write(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - t0) / 1e3:9.1f} "
                         f"{r.get(key, '-') if key else '-':>4} {r.get('Grid_Size', ''):>8} "
                         f"{r['Kernel_Name'].split('(')[0].replace('void ', '')[:90]}\n")
    if key:
        by = defaultdict(list)
        for r in rows[a + 1:b + 1]:
            by[r[key]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
        print(f"per {key}: busy us (kernels)")
        for q, iv in sorted(by.items(), key=lambda kv: -len(kv[1])):
            iv.sort()
            tot, c = 0, t0
            for s0, e0, _ in iv:
                if e0 > c:
                    tot += e0 - max(s0, c)
                    c = e0
            top = defaultdict(float)
            for s0, e0, n in iv:
                top[n.split("(")[0].replace("void ", "")[:40]] += (e0 - s0) / 1e3
            tops = ", ".join(f"{k} {v:.0f}" for k, v in sorted(top.items(), key=lambda kv: -kv[1])[:3])
            print(f"  {q}: {tot / 1e3:8.1f} us ({len(iv)})  {tops}")


if __name__ == "__main__":
    main()
