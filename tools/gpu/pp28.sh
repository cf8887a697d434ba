#!/bin/bash
# padded-width 3x3 wgrad (224x224 widths): tests, per-shape timing, config-5 step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp28; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for sh in 1024,56,56,64,64,3,1,1 1024,28,28,128,128,3,1,1 1024,14,14,256,256,3,1,1 1024,7,7,512,512,3,1,1; do
  for v in 1 0; do echo "pad=$v $sh $(SDX_W3_PAD=$v timeout -k 10 60 python tools/conv_one.py --mode wgrad --shape $sh --iters 20 2>&1 | grep -v amdgpu.ids | tail -n 1)"; done
done | tee $O/shapes.txt
BENCH_ARGS="--config supcon224" bash tools/gpu/ab_bench.sh 2 "pad1:X=1" "pad0:SDX_W3_PAD=0"
