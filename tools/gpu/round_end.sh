# Round-end rehearsal of the driver tiers on the final tree: the whole GPU test tier, smoke(),
# the default bench.py (twice), the end-state step profile and the config-5 bench.
# A crash / timeout ends the script.
set -o pipefail
mkdir -p gpurun_out/r3e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3e/gpu_tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3e/smoke.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > gpurun_out/r3e/bench1.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > gpurun_out/r3e/bench2.txt 2>&1 || exit 1
bash tools/profile_step.sh r3end > gpurun_out/r3e/profile.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config supcon224 --steps 6 --warmup 2 > gpurun_out/r3e/cfg5_bench.txt 2>&1 || exit 1
