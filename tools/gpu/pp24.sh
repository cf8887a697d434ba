#!/bin/bash
# strided 1x1 wgrad on the pipelined kernel + 4-wave 64x128 wave tiles (cfgs 7/8) with VGPR-form MFMA
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp24; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in -1 6 7 8; do timeout -k 10 240 python tools/conv_bench.py --no_miopen --cfg $c > $O/cb_$c.txt 2>&1 || exit 1; done
tail -4 $O/cb_-1.txt $O/cb_6.txt $O/cb_7.txt $O/cb_8.txt
