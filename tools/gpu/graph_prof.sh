#!/bin/bash
# Kernel trace of the hipGraph-replayed step (128 images/GPU, no SyncBN) -> gpurun_out/prof_graph/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/prof_graph
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/pg -o run -- python3 bench.py --per_gpu_batch 128 --graph 1 --steps 10 --warmup 3 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python tools/rocpd_to_csv.py /tmp/pg > /dev/null
d=$(dirname $(find /tmp/pg -name "run_kernel_trace.csv" | head -1))
python tools/step_timeline.py $d --dump $O/step_kernels.txt > $O/timeline.txt
head -40 $O/timeline.txt
