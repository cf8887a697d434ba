# Side-stream wgrad block target (SDX_W3_BLOCKS, default 128) re-tuned with the pipelined 1x1
# kernel: interleaved bench A/B.
set -o pipefail
mkdir -p gpurun_out/r3b
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/ab_bench.sh 3 "b128:" "b96:SDX_W3_BLOCKS=96" "b192:SDX_W3_BLOCKS=192" "b256:SDX_W3_BLOCKS=256" > gpurun_out/r3b/ab.txt 2>&1 || exit 1
