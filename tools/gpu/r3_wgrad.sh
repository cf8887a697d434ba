# Weight-gradient evidence: step profile with per-stream kernel dump, per-dispatch durations of
# every conv kernel over the conv table (wgrad kernel vs split-K reduce), PMC of the 1x1 and
# 3x3 wgrad kernels on layer-3 shapes, and the fused SyncBN exchange at W = 2 (protocol cost
# with only a 2-fold emulated reduction). A crash / timeout ends the script.
set -o pipefail
mkdir -p gpurun_out/r3w
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/profile_step.sh r3b > gpurun_out/r3w/profile.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/cb -o run -- python3 tools/conv_bench.py --no_miopen --iters 10 > gpurun_out/r3w/conv_bench.txt 2>&1 || exit 1
python tools/rocpd_to_csv.py /tmp/cb > /dev/null
d=$(dirname $(find /tmp/cb -name "run_kernel_trace.csv" | head -1))
python tools/kernel_durations.py $d > gpurun_out/r3w/conv_kernels.txt
bash tools/pmc_one.sh w1_l3c1 python3 tools/conv_one.py --mode wgrad --shape 512,8,8,1024,256,1,1,0 --iters 5 > gpurun_out/r3w/pmc1.txt 2>&1 || exit 3
bash tools/pmc_one.sh w3_l3c2 python3 tools/conv_one.py --mode wgrad --shape 512,8,8,256,256,3,1,1 --iters 5 > gpurun_out/r3w/pmc3.txt 2>&1 || exit 3
python tools/pmc_table.py gpurun_out/pmc > gpurun_out/r3w/pmc_table.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/lat1 -o run -- python3 tools/syncbn_latency.py 2 200 > gpurun_out/r3w/lat1.txt 2>&1 || exit 1
python tools/rocpd_to_csv.py /tmp/lat1 > /dev/null
d=$(dirname $(find /tmp/lat1 -name "run_kernel_trace.csv" | head -1))
python tools/kernel_durations.py $d --match col_reduce bn_finalize > gpurun_out/r3w/lat1_kernels.txt
