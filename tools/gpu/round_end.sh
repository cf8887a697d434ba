# Round-end rehearsal of the driver tiers on the final tree: the whole GPU test tier, smoke(),
# the default bench.py (twice), the end-state step profile and the config-5 bench.
# A crash / timeout ends the script.
set -o pipefail
mkdir -p gpurun_out/r4e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4e/gpu_tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4e/smoke.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > gpurun_out/r4e/bench1.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > gpurun_out/r4e/bench2.txt 2>&1 || exit 1
bash tools/profile_step.sh r4end > gpurun_out/r4e/profile.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config supcon224 --steps 6 --warmup 2 > gpurun_out/r4e/cfg5_bench.txt 2>&1 || exit 1
grep -E "passed|failed" gpurun_out/r4e/gpu_tests.txt | tail -n 2; tail -n 1 gpurun_out/r4e/smoke.txt; grep -o "\"ms_per_step\": [0-9.]*" gpurun_out/r4e/bench1.txt gpurun_out/r4e/bench2.txt gpurun_out/r4e/cfg5_bench.txt; head -n 3 gpurun_out/prof_r4end/timeline.txt
