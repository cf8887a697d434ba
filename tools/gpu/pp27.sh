#!/bin/bash
# wgrad kernels: LDS traffic + refill loads issued before the MFMAs (SDX_W_ORDER) and the zero
# page pinned in SGPRs (3x3 kernels): tests, standalone timing, step A/B vs the compiler's order
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp27; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for sh in 512,8,8,1024,256,1,1,0 512,16,16,512,128,1,1,0 512,8,8,256,256,3,1,1 512,16,16,128,128,3,1,1 512,32,32,64,64,3,1,1 512,16,16,256,256,3,2,1; do
  for v in "" wo0; do echo "v=${v:-new} $sh $(SDX_EXT_VARIANT=$v timeout -k 10 60 python tools/conv_one.py --mode wgrad --shape $sh --iters 50 2>&1 | grep -v amdgpu.ids | tail -n 1)"; done
done | tee $O/shapes.txt
bash tools/gpu/ab_bench.sh 3 "new:X=1" "wo0:SDX_EXT_VARIANT=wo0"
