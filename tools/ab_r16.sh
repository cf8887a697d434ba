set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r16
mkdir -p $O
SDX_IGEMM_RING=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/ring_tests.log 2>&1 || { tail -30 $O/ring_tests.log; exit 1; }
tail -2 $O/ring_tests.log
timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb_base.txt 2>&1 || exit 1
SDX_IGEMM_RING=1 timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb_ring.txt 2>&1 || exit 1
tail -3 $O/cb_base.txt; tail -3 $O/cb_ring.txt
for v in base ring prio ringprio; do
  case $v in base) E="";; ring) E="SDX_IGEMM_RING=1";; prio) E="SDX_STREAM_PRIO=1";; ringprio) E="SDX_IGEMM_RING=1 SDX_STREAM_PRIO=1";; esac
  env $E timeout -k 10 150 python bench.py --steps 30 --warmup 10 > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log)"
done
timeout -k 10 400 python tools/wgrad_sweep.py > $O/wsweep.txt 2>&1 || { tail -20 $O/wsweep.txt; exit 1; }
tail -3 $O/wsweep.txt
