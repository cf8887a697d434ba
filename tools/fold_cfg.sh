#!/bin/bash
# BN3 fold eligibility A/B on the GPU box: fold tests, then the headline bench and the
# config-5 slice (224x224, 512 images/GPU) with the rows-per-K² rule (default) vs layers 1-2
# only (SDX_BN3_FOLD_MAXK=128) vs off.  -> gpurun_out/foldcfg/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/foldcfg
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fold or block_pairs" -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/tests.log | tail -30; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for spec in "rule:" "k128:SDX_BN3_FOLD_MAXK=128" "off:SDX_BN3_FOLD=0"; do
  tag=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/${tag}_b256.txt 2>&1 || { tail -5 $O/${tag}_b256.txt; exit 1; }
  env $envs timeout -k 10 300 python bench.py --config supcon224 --steps 4 --warmup 2 > $O/${tag}_cfg5.txt 2>&1 || { tail -5 $O/${tag}_cfg5.txt; exit 1; }
  echo "== $tag: b256 $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_b256.txt)  cfg5 $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_cfg5.txt)"
done
