#!/bin/bash
# In-step A/B of the tap-reuse loop (SDX_TAP3=1 default vs 0), interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/tap3b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tap3.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2 3; do
  for spec in "on:SDX_TAP3=1" "off:SDX_TAP3=0"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/bench_${tag}_$i.txt 2>&1 || { tail -5 $O/bench_${tag}_$i.txt; exit 1; }
    echo "$tag round $i $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${tag}_$i.txt)" | tee -a $O/summary.txt
  done
done
