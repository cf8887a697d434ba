set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pp16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -s -k "dgrad or bn3_fold_full_batch or merged_splitk" > $O/t1.log 2>&1; rc=$?; tail -2 $O/t1.log; grep "worst" $O/t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb.txt 2>&1 || exit 1
SDX_DGRAD_MERGE=0 timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb_nomerge.txt 2>&1 || exit 1
grep "\.0\.\(c2\|sc\) *dgrad" $O/cb.txt $O/cb_nomerge.txt
bash tools/profile_step.sh r4b > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -30 gpurun_out/prof_r4b/summary.txt; head -22 gpurun_out/prof_r4b/timeline.txt
