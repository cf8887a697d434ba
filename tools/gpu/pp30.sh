#!/bin/bash
# strided 1x1 wgrad for any output width (GEN instantiation): tests, config-5 A/B, CIFAR A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp30; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for sh in 1024,56,56,256,512,1,2,0 1024,28,28,512,1024,1,2,0 1024,14,14,1024,2048,1,2,0; do
  for v in 1 0; do echo "st=$v $sh $(SDX_W1_STRIDED=$v timeout -k 10 60 python tools/conv_one.py --mode wgrad --shape $sh --iters 20 2>&1 | grep -v amdgpu.ids | tail -n 1)"; done
done | tee $O/shapes.txt
BENCH_ARGS="--config supcon224" bash tools/gpu/ab_bench.sh 2 "st1:X=1" "st0:SDX_W1_STRIDED=0"
