#!/bin/bash
# Tap-reuse loop: numerics, per-shape config sweep, in-kernel step timelines. -> gpurun_out/tap3s/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/tap3s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tap3.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python tools/tap3_sweep.py > $O/sweep.txt 2>&1 || { tail -5 $O/sweep.txt; exit 1; }
cat $O/sweep.txt
{
for spec in "512,8,8,256,256,3,1,1 12" "512,8,8,256,256,3,1,1 13" "512,32,32,64,64,3,1,1 11" "512,16,16,128,128,3,1,1 13"; do
  set -- $spec
  echo "== trace fwd $1 cfg $2"
  timeout -k 10 60 python tools/igemm_trace.py --mode fwd --shape $1 --cfg $2 2>&1 | grep -v amdgpu.ids || exit 1
done
} > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
grep -E "==|wave 0|K-tiles" $O/trace.txt
