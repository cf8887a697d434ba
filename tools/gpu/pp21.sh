set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
rm -f gpurun_out/ab/summary.txt
bash tools/gpu/ab_bench.sh 3 "m2:X=1" "m1:SDX_DGRAD_MERGE=1" "m0:SDX_DGRAD_MERGE=0" > /dev/null || exit 1
cat gpurun_out/ab/summary.txt
