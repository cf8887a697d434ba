#!/bin/bash
# The whole GPU test tier (stops at the first failure). -> gpurun_out/gt/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${@} > gpurun_out/gt/tests.txt 2>&1; rc=$?
tail -15 gpurun_out/gt/tests.txt
exit $rc
