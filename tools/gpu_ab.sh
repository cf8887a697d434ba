#!/bin/bash
# Quick A/B round on the GPU box after a kernel change: conv numerics (+ fuzz, bounds-checked
# build), per-shape conv table, two bench runs. Extra environment (e.g. SDX_IGEMM_RING=1) is
# passed through. Usage: bash tools/gpu_ab.sh TAG   -> gpurun_out/ab_TAG/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ab_${1:-cur}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fuzz.py tests/test_gpu_checked.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb.txt 2>&1 || exit 1
grep TOTAL $O/cb.txt
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 10 > $O/bench$i.log 2>&1 || { tail -20 $O/bench$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/bench$i.log
done
