#!/usr/bin/env python3
"""Convert a rocprofv3 SQLite result (``*_results.db``, the default output format) into the
CSV files the other tools read: ``<dir>/run_kernel_trace.csv`` (Kernel_Name,
Start_Timestamp, End_Timestamp, VGPR, LDS) and ``<dir>/run_kernel_stats.csv`` (Name, Calls,
TotalDurationNs, AverageNs).

python tools/rocpd_to_csv.py <rocprof output dir>
"""
import csv
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        sys.exit(f"no .db under {d}")
    rows = []
    extra = []
    for db in dbs:
        c = sqlite3.connect(db)
        cols = [x[0] for x in c.execute("select * from kernels limit 1").description]
        # stream / queue ids when the schema has them (per-stream timelines, tools/step_timeline.py)
        extra = [k for k in ("stream_id", "queue_id") if k in cols]
        rows += c.execute("select name, start, end, vgpr_count, accum_vgpr_count, lds_size, grid_x, workgroup_x" +
                          "".join(", " + k for k in extra) + " from kernels order by start").fetchall()
    rows.sort(key=lambda r: r[1])
    with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "VGPR_Count", "Accum_VGPR_Count",
                    "LDS_Block_Size", "Grid_Size", "Workgroup_Size"] +
                   [{"stream_id": "Stream_Id", "queue_id": "Queue_Id"}[k] for k in extra])
        w.writerows(rows)
    agg = defaultdict(lambda: [0, 0])
    for r in rows:
        agg[r[0]][0] += 1
        agg[r[0]][1] += r[2] - r[1]
    with open(os.path.join(d, "run_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs"])
        for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, n, t, t / n])
    print(f"{len(rows)} dispatches -> {d}/run_kernel_{{trace,stats}}.csv")


if __name__ == "__main__":
    main()
