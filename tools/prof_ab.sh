#!/bin/bash
# A/B kernel-time profile of an env toggle on the bench (GPU box):
#   bash tools/prof_ab.sh VAR          -> gpurun_out/sum_VAR_{1,0}.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
VAR=${1:-SDX_DGRAD_BNSTAT}
mkdir -p gpurun_out
for mode in 1 0; do
  env $VAR=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/p$mode -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/p_${VAR}_$mode.log 2>&1 || exit 1
  python tools/rocpd_to_csv.py /tmp/p$mode > /dev/null 2>&1
  f=$(find /tmp/p$mode -name "*kernel_stats.csv" | head -1)
  mkdir -p /tmp/s$mode && cp "$f" /tmp/s$mode/run_kernel_stats.csv
  python tools/rocprof_summary.py /tmp/s$mode --steps 16 > gpurun_out/sum_${VAR}_$mode.txt
done
head -16 gpurun_out/sum_${VAR}_1.txt; head -16 gpurun_out/sum_${VAR}_0.txt
