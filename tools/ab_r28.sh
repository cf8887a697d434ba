set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r28
mkdir -p $O
for g in 0 1 0 1; do
  timeout -k 10 200 python bench.py --graph $g --steps 30 --warmup 10 > $O/b$g.log 2>&1 || { tail -20 $O/b$g.log; exit 1; }
  echo "graph=$g $(grep -o '"ms_per_step": [0-9.]*' $O/b$g.log) $(grep -o '"hip_graph": [a-z]*' $O/b$g.log) $(grep 'host issue' $O/b$g.log | tr '\n' ' ')"
done
