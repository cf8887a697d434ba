#!/bin/bash
# fewer torch kernels in the step: tests, bench, step profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp38; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_supcon.py tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash tools/profile_step.sh r4z > $O/prof.log 2>&1 || { tail -n 20 $O/prof.log; exit 1; }
grep -c "at::native" gpurun_out/prof_r4z/step_kernels.txt; grep "at::native\|rocclr" gpurun_out/prof_r4z/step_kernels.txt | cut -c1-140
