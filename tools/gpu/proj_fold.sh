#!/bin/bash
# Projection-block forward fold: parity tests, then the in-step A/B (with the tile-rule masks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fold" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pf/tests.txt 2>&1 || { tail -30 gpurun_out/pf/tests.txt; exit 1; }
grep -E "worst|passed|failed" gpurun_out/pf/tests.txt | tail -12
bash tools/gpu/ab_env.sh 2 "p1r7:SDX_CFG_RULES=7" "p0r7:SDX_FOLD_FWD_PROJ=0" "p1r0:SDX_CFG_RULES=0" "p1r1:SDX_CFG_RULES=1" "p1r2:SDX_CFG_RULES=2" "p1r4:SDX_CFG_RULES=4"
