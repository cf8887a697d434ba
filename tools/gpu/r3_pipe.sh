# Fragment-pipelined wgrad kernels: wgrad tests, per-dispatch kernel time over the conv table
# with both pipelined kernels (1 1) / only the 1x1 one (1 0) / neither (0 0), bench A/B.
set -o pipefail
mkdir -p gpurun_out/r3q
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -v -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/r3q/tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for v in "1 1" "1 0" "0 0"; do
  set -- $v; t=$1$2
  SDX_W1_PIPE=$1 SDX_W3_PIPE=$2 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cb$t -o run -- python3 tools/conv_bench.py --no_miopen --iters 10 > gpurun_out/r3q/conv_bench_$t.txt 2>&1 || exit 1
  python tools/rocpd_to_csv.py /tmp/cb$t > /dev/null
  d=$(dirname $(find /tmp/cb$t -name "run_kernel_trace.csv" | head -1))
  python tools/kernel_durations.py $d --match wgrad splitk > gpurun_out/r3q/kernels_$t.txt
done
bash tools/gpu/ab_bench.sh 3 "pp:" "p0:SDX_W3_PIPE=0" "00:SDX_W1_PIPE=0 SDX_W3_PIPE=0" > gpurun_out/r3q/ab.txt 2>&1 || exit 1
