#!/bin/bash
# Config-5 (224x224 SupCon, LARS, 512 images x 2 views) per-kernel table: rocprofv3 kernel trace of
# bench.py --config supcon224, summarised per step (steps = wprep_kernel launches, one per step).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/cfg5prof
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/pc5 -o run -- python3 bench.py --config supcon224 --steps 3 --warmup 1 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python tools/rocpd_to_csv.py /tmp/pc5 > /dev/null
d=$(dirname $(find /tmp/pc5 -name "run_kernel_trace.csv" | head -1))
n=$(grep -c "wprep_kernel" $d/run_kernel_trace.csv)
echo "steps (wprep launches): $n"
python tools/rocprof_summary.py $d --steps $((n - 1)) > $O/summary.txt
head -40 $O/summary.txt
