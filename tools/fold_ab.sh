#!/bin/bash
# BN3 fold (csrc/kernels/bnfold.hip) on the GPU box: parity tests (fold vs unfolded, block
# pairs vs fp32 with the fold, head masked-store GEMMs), then the driver bench interleaved
# SDX_BN3_FOLD=0 / 1, and the step profile with the fold on.
# Usage: bash tools/fold_ab.sh  -> gpurun_out/fold/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/fold
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_head.py -k "fold or block_pairs or head" -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
for r in 1 2; do
  for f in 0 1; do
    SDX_BN3_FOLD=$f timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/bench_f${f}_$r.txt 2>&1 || { tail -20 $O/bench_f${f}_$r.txt; exit 1; }
    echo "== fold=$f run $r: $(grep -o '"ms_per_step": [0-9.]*' $O/bench_f${f}_$r.txt) $(grep -o '"last_loss_local": [0-9.]*' $O/bench_f${f}_$r.txt)"
  done
done
