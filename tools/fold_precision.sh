#!/bin/bash
# BN3 fold precision at the headline batch (tests/test_gpu_parity.py::test_bn3_fold_full_batch_gradients)
# with the full coherent-rounding correction (default) and without its mean(a2) part
# (SDX_FOLD_GRAM_FWD=0), then the fold tests and the headline bench fold on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/foldprec
mkdir -p $O
for g in 1 0; do
  SDX_FOLD_GRAM_FWD=$g timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k full_batch -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/full_g$g.log 2>&1
  echo "gram_fwd=$g: $(grep -o 'worst: .*' $O/full_g$g.log) $(grep -oE '[0-9]+ (passed|failed)' $O/full_g$g.log)"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_misc.py -k "fold or block_pairs or graph or engine" -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 0 1; do
  SDX_BN3_FOLD=$f timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/b_f$f.txt 2>&1 || { tail -5 $O/b_f$f.txt; exit 1; }
  echo "== fold=$f: $(grep -o '"ms_per_step": [0-9.]*' $O/b_f$f.txt)"
done
