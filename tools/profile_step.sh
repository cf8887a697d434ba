#!/bin/bash
# Current-state step profile on the GPU box: phase timers (--profile), rocprofv3 kernel
# stats + per-step timeline. Writes gpurun_out/prof_<tag>/{phases.txt,summary.txt,timeline.txt}
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-cur}
O=gpurun_out/prof_$TAG
mkdir -p $O
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --profile > $O/phases.txt 2>&1 || { tail -20 $O/phases.txt; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pp -o run -- python3 bench.py --steps 10 --warmup 3 > /tmp/pp.log 2>&1 || { tail -20 /tmp/pp.log; exit 1; }
python tools/rocpd_to_csv.py /tmp/pp > /dev/null
d=$(dirname $(find /tmp/pp -name "run_kernel_trace.csv" | head -1))
python tools/rocprof_summary.py $d --steps 8 > $O/summary.txt
python tools/step_timeline.py $d --dump $O/step_kernels.txt > $O/timeline.txt
grep -v amdgpu.ids $O/phases.txt | tail -25; head -30 $O/summary.txt; head -12 $O/timeline.txt
