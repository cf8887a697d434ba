set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
rm -f gpurun_out/ab/summary.txt
bash tools/gpu/ab_bench.sh 3 "tail:X=1" "notail:SDX_W3_TAIL_PIX=0" "tail512:SDX_W3_TAIL_BLOCKS=512" > /dev/null || exit 1
cat gpurun_out/ab/summary.txt
bash tools/profile_step.sh r4c > /tmp/prof.log 2>&1 || { tail -20 /tmp/prof.log; exit 1; }
head -16 gpurun_out/prof_r4c/timeline.txt
