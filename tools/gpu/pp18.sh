set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pp18; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -s -k "trajectory_tracks" > $O/t.log 2>&1; rc=$?; grep "window means" $O/t.log; tail -1 $O/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log; grep "host issue" $O/bench.log
SDX_DGRAD_MERGE=0 SDX_SPLITK_MERGE=0 SDX_CONV_D6=0 timeout -k 10 200 python bench.py > $O/bench_r3.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/bench_r3.log
timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb.txt 2>&1 || exit 1
tail -n 4 $O/cb.txt
bash tools/profile_step.sh r4b > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -12 gpurun_out/prof_r4b/summary.txt; head -3 gpurun_out/prof_r4b/timeline.txt
