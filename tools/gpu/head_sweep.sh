#!/bin/bash
# Projection-head GEMM tile sweep (512 rows: 2048->2048 and 2048->128, fwd and dgrad) -> gpurun_out/head/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/head
for shape in 512,1,1,2048,2048,1,1,0 512,1,1,2048,128,1,1,0; do
  for mode in fwd dgrad; do
    for cfg in -1 0 1 2 3 4 5 6; do
      timeout -k 10 60 python tools/conv_one.py --mode $mode --shape $shape --cfg $cfg --iters 50 --nostats 2>/dev/null | grep -v amdgpu || echo "$mode $shape cfg $cfg failed"
    done
  done
done | tee gpurun_out/head/sweep.txt
