#!/bin/bash
# generic wgrad block target (layer-1 1x1 wgrads, stem) re-check
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/ab_bench.sh 2 "t512:X=1" "t256:SDX_WGRAD_TARGET=256" "t128:SDX_WGRAD_TARGET=128"
