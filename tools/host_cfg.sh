# host-side cost of one native step (cProfile + per-phase host times) and config-5 without
# micro-batching. Writes gpurun_out/host/*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/host
mkdir -p $O
timeout -k 10 200 python tools/host_profile.py > $O/cprofile.txt 2>&1 || { tail -20 $O/cprofile.txt; exit 1; }
timeout -k 10 200 python tools/host_phases.py > $O/phases.txt 2>&1 || { tail -20 $O/phases.txt; exit 1; }
timeout -k 10 400 python bench.py --config supcon224 --micro_batch 0 --steps 3 --warmup 1 > $O/cfg5_full.json 2> $O/cfg5_full.err || { tail -20 $O/cfg5_full.err; exit 1; }
tail -1 $O/cfg5_full.json
