#!/bin/bash
# merged SupCon backward (dA + dC in one reduce): tests + step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp37; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_supcon.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?; tail -n 2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 40 --warmup 10 > $O/bench.txt 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*\|"first_loss_local": [0-9.]*\|"last_loss_local": [0-9.]*' $O/bench.txt
