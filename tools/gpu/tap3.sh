#!/bin/bash
# Tap-reuse 3x3 loop: numerics (new + existing conv tests), per-shape conv table with the loop
# on / off, interleaved driver-bench A/B. -> gpurun_out/tap3/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/tap3
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tap3.py > $O/tests_tap3.txt 2>&1 || { tail -30 $O/tests_tap3.txt; exit 1; }
tail -3 $O/tests_tap3.txt
timeout -k 10 200 python tools/conv_bench.py --no_miopen --iters 30 > $O/cb_on.txt 2>&1 || { tail -5 $O/cb_on.txt; exit 1; }
SDX_TAP3=0 timeout -k 10 200 python tools/conv_bench.py --no_miopen --iters 30 > $O/cb_off.txt 2>&1 || { tail -5 $O/cb_off.txt; exit 1; }
grep TOTAL $O/cb_on.txt $O/cb_off.txt
for i in 1 2; do
  for spec in "on:SDX_TAP3=1" "off:SDX_TAP3=0"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/bench_${tag}_$i.txt 2>&1 || { tail -5 $O/bench_${tag}_$i.txt; exit 1; }
    echo "$tag round $i $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${tag}_$i.txt)" | tee -a $O/summary.txt
  done
done
