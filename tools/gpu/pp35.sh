#!/bin/bash
# strided 3x3 dgrad (merged sub-pixel classes): tile config sweep
cd "${GRAFT_REPO_ROOT:-.}"
for sh in 512,32,32,128,128,3,2,1 512,16,16,256,256,3,2,1 512,8,8,512,512,3,2,1; do
  for c in -1 0 1 2 3 4 5 6; do
    echo "$sh cfg $c: $(timeout -k 10 60 python tools/conv_one.py --mode dgrad --shape $sh --cfg $c --iters 30 2>&1 | grep -v amdgpu.ids | tail -n 1)"
  done
done | tee gpurun_out/pp35.txt
