#!/bin/bash
# BN3 fold with the addend added before rounding (variant build: csrc/build.py --variant addpre
# --define SDX_ADD_PRE=1): precision probe + full-batch test + fold tests on the variant, then the
# headline bench: variant fold on / base fold on / fold off.  -> gpurun_out/addpre/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/addpre
mkdir -p $O
SDX_EXT_VARIANT=addpre timeout -k 10 400 python tools/fold_bn_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -E "pair|bn2" $O/probe.txt
SDX_EXT_VARIANT=addpre timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fold or block_pairs" -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
grep -E "worst|PASSED|FAILED|XPASS|XFAIL|passed|failed" $O/tests.log | tail -12
for spec in "var:SDX_EXT_VARIANT=addpre SDX_BN3_FOLD=1" "base:SDX_BN3_FOLD=1" "off:SDX_BN3_FOLD=0"; do
  tag=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/b_$tag.txt 2>&1 || { tail -5 $O/b_$tag.txt; exit 1; }
  echo "== $tag: $(grep -o '"ms_per_step": [0-9.]*' $O/b_$tag.txt)"
done
