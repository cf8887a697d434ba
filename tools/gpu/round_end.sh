#!/bin/bash
# Round-end rehearsal of the driver tiers on the final tree: the whole GPU test tier, smoke(),
# the default bench.py (twice), the end-state step profile and the config-5 bench.
# A crash / timeout ends the script. Usage: bash tools/gpu/round_end.sh TAG -> gpurun_out/TAG/
set -o pipefail
TAG=${1:-re}
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
grep -E "passed|failed" $O/gpu_tests.txt | tail -n 2
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py > $O/bench1.txt 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 40 --warmup 10 > $O/bench2.txt 2>&1 || exit 1
# hipGraph replay of the same step (captured as one chain) and its ratio to eager
timeout -k 10 200 python -u bench.py --graph 1 --steps 40 --warmup 10 > $O/bench_graph.txt 2>&1 || exit 1
python - $O/bench2.txt $O/bench_graph.txt <<'PY' | tee $O/graph_ratio.txt
import json, sys
e, g = (json.loads([l for l in open(f) if l.startswith('{"metric"')][0]) for f in sys.argv[1:3])
print(f"graph/eager: {g['ms_per_step']} / {e['ms_per_step']} ms = {g['ms_per_step'] / e['ms_per_step']:.3f} (hip_graph={g['config']['hip_graph']})")
PY
bash tools/profile_step.sh ${TAG}p > $O/profile.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --config supcon224 --steps 6 --warmup 2 > $O/cfg5_bench.txt 2>&1 || exit 1
tail -n 1 $O/smoke.txt; grep -o "\"ms_per_step\": [0-9.]*" $O/bench1.txt $O/bench2.txt $O/cfg5_bench.txt; head -n 3 gpurun_out/prof_${TAG}p/timeline.txt
