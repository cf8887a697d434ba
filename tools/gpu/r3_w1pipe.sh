# Fragment-pipelined 1x1 wgrad kernel: correctness (wgrad tests), per-dispatch kernel time over the conv
# table vs the register-staged kernel (SDX_W1_PIPE=0), and the bench step A/B.
set -o pipefail
mkdir -p gpurun_out/r3p
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -v -k "wgrad" --timeout 120 --timeout-method thread > gpurun_out/r3p/tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
for v in 1 0; do
  SDX_W1_PIPE=$v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cb$v -o run -- python3 tools/conv_bench.py --no_miopen --iters 10 > gpurun_out/r3p/conv_bench_$v.txt 2>&1 || exit 1
  python tools/rocpd_to_csv.py /tmp/cb$v > /dev/null
  d=$(dirname $(find /tmp/cb$v -name "run_kernel_trace.csv" | head -1))
  python tools/kernel_durations.py $d --match wgrad splitk > gpurun_out/r3p/kernels_$v.txt
done
bash tools/gpu/ab_bench.sh 3 "pipe:" "reg:SDX_W1_PIPE=0" > gpurun_out/r3p/ab.txt 2>&1 || exit 1
