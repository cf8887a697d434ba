#!/bin/bash
# config 5 (supcon224): side-stream wgrad block targets
cd "${GRAFT_REPO_ROOT:-.}"
BENCH_ARGS="--config supcon224" bash tools/gpu/ab_bench.sh 2 "base:X=1" "b256:SDX_W3_BLOCKS=256" "t1024:SDX_WGRAD_TARGET=1024" "both:SDX_W3_BLOCKS=256 SDX_WGRAD_TARGET=1024"
