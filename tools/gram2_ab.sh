#!/bin/bash
# With the accumulator pre-add in place: forward-time Grams (SDX_FOLD_GRAM_FWD=1, feeds the mean(a2)
# part of the bias correction) vs Grams in backward (0): full-batch fold precision test and the
# headline bench interleaved.  -> gpurun_out/gram2/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/gram2
mkdir -p $O
SDX_FOLD_GRAM_FWD=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k full_batch -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/full_g0.log 2>&1
echo "gram_fwd=0 full batch: $(grep -o 'worst: .*' $O/full_g0.log) $(grep -oE '[0-9]+ (passed|failed)' $O/full_g0.log)"
for r in 1 2; do
  for g in 1 0; do
    SDX_FOLD_GRAM_FWD=$g timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/b_g${g}_$r.txt 2>&1 || { tail -5 $O/b_g${g}_$r.txt; exit 1; }
    echo "== gram_fwd=$g run $r: $(grep -o '"ms_per_step": [0-9.]*' $O/b_g${g}_$r.txt)"
  done
done
