#!/bin/bash
# end-state per-shape conv table (auto configs, MIOpen columns included)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp34; mkdir -p $O
timeout -k 10 400 python tools/conv_bench.py > $O/cb.txt 2>&1 || { tail -n 5 $O/cb.txt; exit 1; }
tail -n 4 $O/cb.txt
