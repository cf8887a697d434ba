#!/bin/bash
# eager vs whole-step hipGraph bench (alternating), then the current step profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/graph
for g in 0 1 0 1; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 10 --graph $g > gpurun_out/graph/g$g.txt 2>&1 || { tail -5 gpurun_out/graph/g$g.txt; exit 1; }
  echo "graph=$g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/graph/g$g.txt) $(grep -o '"hip_graph": [a-z]*' gpurun_out/graph/g$g.txt)"
done
bash tools/profile_step.sh r2b > /dev/null 2>&1 || exit 1
head -30 gpurun_out/prof_r2b/summary.txt; head -3 gpurun_out/prof_r2b/timeline.txt
