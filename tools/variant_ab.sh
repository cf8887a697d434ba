#!/bin/bash
# A/B of experiment builds (csrc/build.py --variant V --define ...): per-shape conv table and
# the driver bench for the base build and each variant. Build the variants on the CPU first.
# Usage: bash tools/variant_ab.sh V1 [V2 ...]   -> gpurun_out/vab/{base,V1,...}_{cb,bench}.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/vab
mkdir -p $O
for v in base "$@"; do
  if [ "$v" = base ]; then unset SDX_EXT_VARIANT; else export SDX_EXT_VARIANT=$v; fi
  timeout -k 10 200 python tools/conv_bench.py --no_miopen --iters 30 > $O/${v}_cb.txt 2>&1 || { tail -20 $O/${v}_cb.txt; exit 1; }
  timeout -k 10 150 python bench.py --steps 30 --warmup 10 > $O/${v}_bench.txt 2>&1 || { tail -20 $O/${v}_bench.txt; exit 1; }
  echo "== $v: $(grep -o '"ms_per_step": [0-9.]*' $O/${v}_bench.txt)"
  grep TOTAL $O/${v}_cb.txt
done
