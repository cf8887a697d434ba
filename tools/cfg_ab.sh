#!/bin/bash
# conv tile-config A/B on the GPU box: tools/conv_bench.py totals for the auto choice, the
# 256x128 8-wave tile, and the 3-buffer LDS-DMA ring (SDX_IGEMM_RING=1) on cfg 0/4/5.
# Result: profiles/conv_cfg_ring_ab_r2.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/cfgab
mkdir -p $O
for spec in "auto:-1:0" "c5:5:0" "c5ring:5:1" "c4ring:4:1" "c0ring:0:1"; do
  IFS=: read tag cfg ring <<< "$spec"
  SDX_IGEMM_RING=$ring timeout -k 10 200 python tools/conv_bench.py --no_miopen --iters 30 --cfg $cfg > $O/$tag.txt 2>&1 || { tail -5 $O/$tag.txt; exit 1; }
  echo "== $tag"; grep TOTAL $O/$tag.txt
done
