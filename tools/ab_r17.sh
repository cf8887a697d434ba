set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/conv_bench.py --no_miopen > $O/cb.txt 2>&1 || exit 1
grep TOTAL $O/cb.txt
bash tools/profile_step.sh v16 > /dev/null 2>&1 || exit 1
SDX_WGRAD_STREAM=0 bash tools/profile_step.sh v16serial > /dev/null 2>&1 || exit 1
grep ms_per_step gpurun_out/prof_v16/phases.txt | grep -o '"ms_per_step": [0-9.]*'
grep ms_per_step gpurun_out/prof_v16serial/phases.txt | grep -o '"ms_per_step": [0-9.]*'
