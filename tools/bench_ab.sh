#!/bin/bash
# Interleaved wall-clock A/B of an env toggle on bench.py (GPU box), R rounds:
#   bash tools/bench_ab.sh VAR [R] [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
VAR=${1:-SDX_DGRAD_BNSTAT}; R=${2:-3}; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for mode in 1 0; do
    env $VAR=$mode timeout -k 10 150 python bench.py --steps 30 --warmup 10 "$@" > /tmp/b.log 2>&1 || { tail -20 /tmp/b.log; exit 1; }
    echo "$VAR=$mode $(grep -o '"ms_per_step": [0-9.]*' /tmp/b.log)" | tee -a gpurun_out/bench_ab_$VAR.txt
  done
done
