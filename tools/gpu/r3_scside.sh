# Shortcut conv on the side stream in the forward (projection blocks): tests, bench A/B
# (SDX_SC_SIDE=0 disables it from Python). Crash / timeout ends it.
set -o pipefail
mkdir -p gpurun_out/r3c gpurun_out/r3r
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_comm.py tests/test_gpu_misc.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > gpurun_out/r3c/tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
bash tools/gpu/ab_bench.sh 3 "side:" "main:SDX_SC_SIDE=0" > gpurun_out/r3c/ab.txt 2>&1 || exit 1
