#!/bin/bash
# A/B of the BatchNorm elementwise unroll (SDX_EW_UNROLL) on the GPU box: BN kernel tests on
# the base build, tools/bn_bench.py per build, then the driver bench interleaved.
# Build the variants on the CPU first:
#   python csrc/build.py --variant ew1 --define SDX_EW_UNROLL=1   (and ew2 ... as wanted)
# Usage: bash tools/ew_ab.sh V1 [V2 ...]   -> gpurun_out/ewab/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ewab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in base "$@"; do
  if [ "$v" = base ]; then unset SDX_EXT_VARIANT; else export SDX_EXT_VARIANT=$v; fi
  timeout -k 10 200 python tools/bn_bench.py > $O/${v}_bn.txt 2>&1 || { tail -20 $O/${v}_bn.txt; exit 1; }
done
for r in 1 2; do
  for v in base "$@"; do
    if [ "$v" = base ]; then unset SDX_EXT_VARIANT; else export SDX_EXT_VARIANT=$v; fi
    timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/${v}_bench$r.txt 2>&1 || { tail -20 $O/${v}_bench$r.txt; exit 1; }
    echo "== $v run $r: $(grep -o '"ms_per_step": [0-9.]*' $O/${v}_bench$r.txt)"
  done
done
