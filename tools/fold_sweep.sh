set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fold2
for r in 1 2; do
for spec in "f0:SDX_BN3_FOLD=0" "k128:SDX_BN3_FOLD=1" "k256:SDX_BN3_FOLD=1 SDX_BN3_FOLD_MAXK=256" "k512:SDX_BN3_FOLD=1 SDX_BN3_FOLD_MAXK=512"; do
  tag=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 10 > gpurun_out/fold2/${tag}_$r.txt 2>&1 || { tail -5 gpurun_out/fold2/${tag}_$r.txt; exit 1; }
  echo "== $tag run $r: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fold2/${tag}_$r.txt)"
done
done
SDX_BN3_FOLD=1 bash tools/profile_step.sh fold > /dev/null 2>&1 || { echo profile failed; exit 1; }
head -45 gpurun_out/prof_fold/summary.txt
