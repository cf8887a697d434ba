#!/bin/bash
# 64-channel 1x1 wgrads on the pixel-pair view: kernel tests, per-shape timing, in-step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/w1p
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -k "wgrad1x1 or sink_accumulate" -x -q --timeout 120 --timeout-method thread > gpurun_out/w1p/tests.txt 2>&1 || { tail -30 gpurun_out/w1p/tests.txt; exit 1; }
tail -2 gpurun_out/w1p/tests.txt
for v in "off:SDX_W1_PAIRS=0" "b256:SDX_W1_PAIR_BLOCKS=256" "b512:SDX_W1_PAIR_BLOCKS=512" "b1024:SDX_W1_PAIR_BLOCKS=1024"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 200 python tools/conv_bench.py --no_miopen > gpurun_out/w1p/cb_$tag.txt 2>&1 || exit 1
  grep -E "l1\..*c[13] .*wgrad|l1\..*sc .*wgrad" gpurun_out/w1p/cb_$tag.txt | sed "s/^/$tag /"
done
bash tools/gpu/ab_env.sh 2 "off:SDX_W1_PAIRS=0" "b256:SDX_W1_PAIR_BLOCKS=256" "b512:SDX_W1_PAIR_BLOCKS=512"
