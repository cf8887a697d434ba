#!/bin/bash
# One build -> measure iteration on the GPU box: the given GPU test files, smoke(), the
# driver-default bench and the step profile (tools/profile_step.sh).
# Usage: bash tools/gpu_iter.sh TAG [test files...]   -> gpurun_out/it_TAG/, gpurun_out/prof_TAG/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${1:-cur}; shift
O=gpurun_out/it_$TAG
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
bash tools/profile_step.sh $TAG > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
head -25 gpurun_out/prof_$TAG/summary.txt; head -8 gpurun_out/prof_$TAG/timeline.txt
