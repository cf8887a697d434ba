#!/bin/bash
# stride-2 3x3 wgrad on padded output rows (224x224 widths 28/14/7): tests, config-5 A/B, CIFAR check
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp31; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for sh in 1024,56,56,128,128,3,2,1 1024,28,28,256,256,3,2,1 1024,14,14,512,512,3,2,1; do
  for v in 1 0; do echo "s2=$v $sh $(SDX_W3_S2=$v timeout -k 10 60 python tools/conv_one.py --mode wgrad --shape $sh --iters 20 2>&1 | grep -v amdgpu.ids | tail -n 1)"; done
done | tee $O/shapes.txt
BENCH_ARGS="--config supcon224" bash tools/gpu/ab_bench.sh 2 "p1:X=1" "p0:SDX_W3_S2=0"
