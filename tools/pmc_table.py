#!/usr/bin/env python3
"""Summarise tools/pmc_report.sh output: per (run, kernel) the mean of each counter over the
kernel's dispatches, plus derived ratios (MFMA busy %, VALU per MFMA, LDS conflict %)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    data = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        run = os.path.relpath(f, root).split(os.sep)[0].rsplit(".", 1)[0]
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not any(t in k for t in ("igemm", "supcon", "splitk", "col_reduce", "wgrad")):
                continue
            name = k.split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
            name = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
            data[(run, name)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for (run, name), c in sorted(data.items()):
        m = {k: sum(v) / len(v) for k, v in c.items()}
        line = f"{run:18s} {name:60s}"
        if "SQ_BUSY_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m and m["SQ_BUSY_CYCLES"]:
            line += f" mfma_busy/busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / m['SQ_BUSY_CYCLES']:.2f}"
        if "SQ_INSTS_VALU" in m and m.get("SQ_INSTS_MFMA"):
            line += f" valu/mfma={m['SQ_INSTS_VALU'] / m['SQ_INSTS_MFMA']:.2f}"
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            line += f" lds_conflict={100 * m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.1f}%"
        if "TCC_HIT_sum" in m and (m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0)):
            line += f" L2_hit={100 * m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m.get('TCC_MISS_sum', 0)):.0f}%"
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            w = m["SQ_WAVE_CYCLES"]
            line += (f" wait_any={100 * m.get('SQ_WAIT_ANY', 0) / w:.0f}% wait_inst={100 * m.get('SQ_WAIT_INST_ANY', 0) / w:.0f}%"
                     f" active={100 * m.get('SQ_ACTIVE_INST_ANY', 0) / w:.0f}%")
        print(line)
        print("    " + " ".join(f"{k}={v:.3g}" for k, v in sorted(m.items())))


if __name__ == "__main__":
    main()
