set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gt_v17.log 2>&1 || { tail -30 gpurun_out/gt_v17.log; exit 1; }
tail -1 gpurun_out/gt_v17.log
bash tools/profile_step.sh v17 > /dev/null 2>&1 || exit 1
SDX_WGRAD_STREAM=0 bash tools/profile_step.sh v17serial > /dev/null 2>&1 || exit 1
timeout -k 10 150 python bench.py > gpurun_out/bench_v17.log 2>&1 || exit 1
tail -1 gpurun_out/bench_v17.log
