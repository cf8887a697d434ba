#!/bin/bash
# 128 vs 256 images/GPU step time (host-bound check) + a kernel timeline
# of the 128/GPU step: idle gaps = the GPU waiting on host issue. -> gpurun_out/b128/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/b128
timeout -k 10 200 python bench.py --per_gpu_batch 128 --steps 30 --warmup 10 > gpurun_out/b128/bench128.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 30 --warmup 10 > gpurun_out/b128/bench256.txt 2>&1 || exit 1
grep -h "host issue\|ms_per_step" gpurun_out/b128/bench128.txt gpurun_out/b128/bench256.txt | sed 's/"metric.*"ms_per_step"/ms_per_step/; s/, "higher.*//'
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pp -o run -- python3 bench.py --per_gpu_batch 128 --steps 10 --warmup 3 > /tmp/pp.log 2>&1 || exit 1
python tools/rocpd_to_csv.py /tmp/pp > /dev/null
d=$(dirname $(find /tmp/pp -name "run_kernel_trace.csv" | head -1))
python tools/step_timeline.py $d > gpurun_out/b128/timeline.txt
head -3 $d/run_kernel_trace.csv | cut -c1-400 > gpurun_out/b128/cols.txt
cat gpurun_out/b128/timeline.txt | tail -12
