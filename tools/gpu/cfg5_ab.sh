#!/bin/bash
# Config-5 (224x224 SupCon, LARS) bench A/B over env settings: bash tools/gpu/cfg5_ab.sh ROUNDS "TAG:ENV=v" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/cfg5ab
mkdir -p $O
R=$1; shift
for i in $(seq 1 $R); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 300 python bench.py --config supcon224 --steps 6 --warmup 2 > $O/${tag}_$i.txt 2>&1 || { tail -5 $O/${tag}_$i.txt; exit 1; }
    echo "$tag round $i $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_$i.txt)" | tee -a $O/summary.txt
  done
done
