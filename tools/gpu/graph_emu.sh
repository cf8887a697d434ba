#!/bin/bash
# Eager vs hipGraph step at 128 and 256 images/GPU with SyncBN over 8 emulated ranks (fused
# exchange, device epochs) and without SyncBN: the host-issue-bound regime of BASELINE
# configs 3/4 (128 images/GPU). -> gpurun_out/graphemu/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/graphemu
mkdir -p $O
for b in 128 256; do
  for g in 0 1; do
    for emu in 0 8; do
      tag=b${b}_g${g}_emu${emu}
      SDX_SYNCBN_EMU=$emu timeout -k 10 200 python bench.py --per_gpu_batch $b --graph $g --steps 40 --warmup 10 > $O/$tag.txt 2>&1 || { tail -5 $O/$tag.txt; exit 1; }
      echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.txt) $(grep -o '"hip_graph": [a-z]*' $O/$tag.txt) $(grep 'idle queue' $O/$tag.txt)" | tee -a $O/summary.txt
    done
  done
done
