# Index-based max-pool backward: tests (pool, config-5 engine step), config-5 bench and
# its per-kernel profile. A crash / timeout ends the script.
set -o pipefail
mkdir -p gpurun_out/r3m
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_misc.py -v -k "maxpool or imagenet" --timeout 300 --timeout-method thread > gpurun_out/r3m/tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config supcon224 --steps 6 --warmup 2 > gpurun_out/r3m/cfg5_bench.txt 2>&1 || exit 1
cd /tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc5 -o run -- python3 bench.py --config supcon224 --steps 4 --warmup 2 > gpurun_out/r3m/cfg5_prof.log 2>&1 || exit 1
python tools/rocpd_to_csv.py /tmp/pc5 > /dev/null
d=$(dirname $(find /tmp/pc5 -name "run_kernel_trace.csv" | head -1))
python tools/rocprof_summary.py $d --steps 9 > gpurun_out/r3m/cfg5_summary.txt
