#!/bin/bash
# strided 1x1 wgrad on the pipelined kernel vs the generic kernel, in the step
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/ab_bench.sh 3 "s1:X=1" "s0:SDX_W1_STRIDED=0"
