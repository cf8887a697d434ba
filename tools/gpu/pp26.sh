#!/bin/bash
# stride-2 tap-reuse 3x3 wgrad: tests, per-shape timing, step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp26; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for sh in 512,32,32,128,128,3,2,1 512,16,16,256,256,3,2,1 512,8,8,512,512,3,2,1; do
  for v in 1 0; do echo "s2=$v $sh $(SDX_W3_S2=$v timeout -k 10 60 python tools/conv_one.py --mode wgrad --shape $sh --iters 50 2>&1 | grep -v amdgpu.ids | tail -n 1)"; done
done | tee $O/shapes.txt
bash tools/gpu/ab_bench.sh 3 "w1:X=1" "w0:SDX_W3_S2=0"
