#!/bin/bash
# Interleaved same-box A/B of the driver bench over env settings, then the conv tests that the
# settings touch. Usage: bash tools/gpu/ab_env.sh ROUNDS "TAG:ENV=v ..." ... -> gpurun_out/abenv/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/abenv
mkdir -p $O
R=$1; shift
for i in $(seq 1 $R); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/${tag}_$i.txt 2>&1 || { tail -5 $O/${tag}_$i.txt; exit 1; }
    echo "$tag round $i $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_$i.txt)" | tee -a $O/summary.txt
  done
done
