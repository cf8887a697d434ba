# Interleaved same-box A/B of the driver bench: bash tools/gpu/ab_bench.sh ROUNDS "TAG:ENV=v ..." ...
# (SDX_EXT_VARIANT=V selects a csrc/build.py --variant build; BENCH_ARGS adds bench.py flags,
# e.g. BENCH_ARGS="--graph 1"). Prints ms/step and the host issue times. -> gpurun_out/ab/summary.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/ab
mkdir -p $O
R=$1; shift
for i in $(seq 1 $R); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 $BENCH_ARGS > $O/${tag}_$i.txt 2>&1 || { tail -5 $O/${tag}_$i.txt; exit 1; }
    echo "$tag round $i $(grep -o '"ms_per_step": [0-9.]*' $O/${tag}_$i.txt) | $(grep -o 'host issue time[^0-9]*[0-9.]*' $O/${tag}_$i.txt | tr '\n' ' ')" | tee -a $O/summary.txt
  done
done
