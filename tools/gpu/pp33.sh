#!/bin/bash
# side-stream wgrad block target re-check with the round-4 wgrad kernels
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/ab_bench.sh 2 "b128:X=1" "b96:SDX_W3_BLOCKS=96" "b160:SDX_W3_BLOCKS=160" "b192:SDX_W3_BLOCKS=192"
