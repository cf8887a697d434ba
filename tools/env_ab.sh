#!/bin/bash
# Environment-toggle A/B on the GPU box: conv_bench totals + the driver bench per setting.
# Usage: bash tools/env_ab.sh "TAG1:VAR=v VAR2=w" "TAG2:VAR=x" ...   (TAG base = no extra env)
# -> gpurun_out/envab/<TAG>_{cb,bench}.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/envab
mkdir -p $O
for spec in "base:" "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python tools/conv_bench.py --no_miopen --iters 30 > $O/${tag}_cb.txt 2>&1 || { tail -5 $O/${tag}_cb.txt; exit 1; }
  env $envs timeout -k 10 150 python bench.py --steps 30 --warmup 10 > $O/${tag}_bench.txt 2>&1 || { tail -5 $O/${tag}_bench.txt; exit 1; }
  echo "== $tag ($envs): $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_bench.txt)"; grep TOTAL $O/${tag}_cb.txt | awk "{print \$2, \$4}" || true
done
