set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pp11; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -s -k "four_rank or test_gpu_conv" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; grep -a "W=4\|hashes" $O/tests.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log; grep "host issue" $O/bench.log
SDX_CONV_D6=0 timeout -k 10 200 python bench.py > $O/bench_nod6.log 2>&1 || exit 1
tail -1 $O/bench_nod6.log | grep -o '"ms_per_step": [0-9.]*'
