#!/bin/bash
# Forward-time fold Grams (SDX_FOLD_GRAM_FWD) on the GPU box: fold / graph / 2-rank tests,
# then the headline bench and the config-5 slice interleaved 0 / 1.  -> gpurun_out/gram/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/gram
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_misc.py tests/test_gpu_dist.py -k "fold or block_pairs or graph or engine or dist or rank" -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for r in 1 2; do
  for g in 0 1; do
    SDX_FOLD_GRAM_FWD=$g timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/b256_g${g}_$r.txt 2>&1 || { tail -5 $O/b256_g${g}_$r.txt; exit 1; }
    echo "== gram_fwd=$g run $r: b256 $(grep -o '"ms_per_step": [0-9.]*' $O/b256_g${g}_$r.txt)"
  done
done
for g in 0 1; do
  SDX_FOLD_GRAM_FWD=$g timeout -k 10 300 python bench.py --config supcon224 --steps 4 --warmup 2 > $O/cfg5_g$g.txt 2>&1 || { tail -5 $O/cfg5_g$g.txt; exit 1; }
  echo "== gram_fwd=$g: cfg5 $(grep -o '"ms_per_step": [0-9.]*' $O/cfg5_g$g.txt)"
done
