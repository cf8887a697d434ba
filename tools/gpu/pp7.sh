set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fwd or dgrad" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 6 5 7; do timeout -k 10 60 python tools/igemm_trace.py --cfg $c > $O/trace_$c.txt 2>&1 || exit 1; done
head -8 $O/trace_6.txt; head -4 $O/trace_7.txt
bash tools/gpu/ablate_conv.sh fwd 512,8,8,256,256,3,1,1 "4 6 5 7" "0 2" > $O/abl.txt 2>&1; cat $O/abl.txt
for c in -1 5 6; do timeout -k 10 200 python tools/conv_bench.py --no_miopen --cfg $c > $O/cb_$c.txt 2>&1 || exit 1; done
