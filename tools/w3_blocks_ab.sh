set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/w3
for r in 1 2; do
for b in 128 96 160 192; do
  SDX_W3_BLOCKS=$b timeout -k 10 150 python bench.py --steps 40 --warmup 10 > gpurun_out/w3/b${b}_$r.txt 2>&1 || { tail -5 gpurun_out/w3/b${b}_$r.txt; exit 1; }
  echo "== W3_BLOCKS=$b run $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/w3/b${b}_$r.txt)"
done
done
