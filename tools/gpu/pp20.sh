set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pp20; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "dgrad" > $O/t.log 2>&1; rc=$?; tail -1 $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb.txt 2>&1 || exit 1
SDX_DGRAD_MERGE=0 timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb0.txt 2>&1 || exit 1
grep -E "\.0\.(c2|sc) +dgrad" $O/cb.txt $O/cb0.txt
rm -f gpurun_out/ab/summary.txt
bash tools/gpu/ab_bench.sh 3 "merge:X=1" "nomerge:SDX_DGRAD_MERGE=0" > /dev/null || exit 1
cat gpurun_out/ab/summary.txt
