set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fwd or dgrad" > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 python tools/igemm_trace.py --cfg 6 2>&1 | grep -v amdgpu.ids | head -4
for c in -1 5 6; do timeout -k 10 200 python tools/conv_bench.py --no_miopen --cfg $c > $O/cb_$c.txt 2>&1 || exit 1; done
tail -3 $O/cb_-1.txt $O/cb_5.txt $O/cb_6.txt
