#!/bin/bash
# K-concatenated BN3-fold dgrad: kernel + fold parity tests, in-step A/B, then the config-5
# A/B of the pixel-pair 1x1 wgrads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fc
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -k "dgrad_cat or fold" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/fc/tests.txt 2>&1 || { grep -E "FAIL|Error|error" gpurun_out/fc/tests.txt | head -20; tail -30 gpurun_out/fc/tests.txt; exit 1; }
grep -E "worst|passed|failed" gpurun_out/fc/tests.txt | tail -12
bash tools/gpu/ab_env.sh 2 "cat1:SDX_FOLD_CAT=1" "cat0:SDX_FOLD_CAT=0"
bash tools/gpu/cfg5_ab.sh 1 "pairs1:SDX_W1_PAIRS=1" "pairs0:SDX_W1_PAIRS=0"
