#!/bin/bash
# Cost of compiling the fold's accumulator pre-add into the dgrad kernels: fold off with the
# default build vs a build without it (csrc/build.py --variant nopre --define SDX_ADD_PRE=0),
# and fold on with the default build, interleaved.  -> gpurun_out/precost/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/precost
mkdir -p $O
for r in 1 2; do
  for spec in "off_pre:SDX_BN3_FOLD=0" "off_nopre:SDX_BN3_FOLD=0 SDX_EXT_VARIANT=nopre" "on_pre:SDX_BN3_FOLD=1"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 > $O/${tag}_$r.txt 2>&1 || { tail -5 $O/${tag}_$r.txt; exit 1; }
    echo "== $tag run $r: $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_$r.txt)"
  done
done
