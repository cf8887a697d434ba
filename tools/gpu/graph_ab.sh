#!/bin/bash
# Eager vs hipGraph replay of the default step at 256 and 128 images/GPU (no SyncBN), the
# graph captured as one chain (default) or with the wgrad side-stream fork kept
# (SDX_GRAPH_SIDE=1). -> gpurun_out/graphab/summary.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/graphab
mkdir -p $O
for b in 256 128; do
  for mode in g0 g1 g1side; do
    g=1; side=0
    [ $mode = g0 ] && g=0
    [ $mode = g1side ] && side=1
    [ $mode = g1side ] && [ $b = 128 ] && continue
    tag=b${b}_${mode}
    SDX_GRAPH_SIDE=$side timeout -k 10 200 python bench.py --per_gpu_batch $b --graph $g --steps 40 --warmup 10 > $O/$tag.txt 2>&1 || { tail -5 $O/$tag.txt; exit 1; }
    echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.txt) $(grep -o '"hip_graph": [a-z]*' $O/$tag.txt) $(grep 'idle queue' $O/$tag.txt)" | tee -a $O/summary.txt
  done
done
