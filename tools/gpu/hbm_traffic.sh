# Per-kernel HBM traffic of the bench step: two counter passes (FETCH_SIZE, WRITE_SIZE) + the
# kernel-trace summary -> gpurun_out/hbm/traffic.txt (tools/hbm_traffic.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/hbm
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d /tmp/hbm_$c -o run -- python3 bench.py --steps 3 --warmup 1 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
done
bash tools/profile_step.sh hbm > /dev/null 2>&1 || exit 1
python tools/hbm_traffic.py /tmp/hbm_FETCH_SIZE /tmp/hbm_WRITE_SIZE gpurun_out/prof_hbm/summary.txt > $O/traffic.txt
head -45 $O/traffic.txt
