#!/bin/bash
# round-4 state: CIFAR step profile + config-5 (supcon224) bench and kernel table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pp22
mkdir -p $O
timeout -k 10 200 bash tools/profile_step.sh r4a > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
timeout -k 10 240 python bench.py --config supcon224 --steps 10 --warmup 3 > $O/c5.txt 2>&1 || { tail -20 $O/c5.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p5 -o run -- python3 bench.py --config supcon224 --steps 4 --warmup 2 > /tmp/p5.log 2>&1 || { tail -20 /tmp/p5.log; exit 1; }
python tools/rocpd_to_csv.py /tmp/p5 > /dev/null
d=$(dirname $(find /tmp/p5 -name "run_kernel_trace.csv" | head -1))
python tools/rocprof_summary.py $d --steps 6 > $O/c5_summary.txt
tail -3 $O/c5.txt; head -30 $O/c5_summary.txt
