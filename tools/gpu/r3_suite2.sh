# Whole GPU test tier after the round-3 kernel changes, PMC passes of the conv main loops
# (fwd / dgrad l3 3x3, fwd l1 1x1 expand) and the pipelined 1x1 wgrad, and the 128-image
# step eager vs hipGraph. A crash / timeout ends the script.
set -o pipefail
mkdir -p gpurun_out/r3s
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3s/gpu_tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
bash tools/pmc_one.sh fwd_l3c2 python3 tools/conv_one.py --mode fwd --shape 512,8,8,256,256,3,1,1 --iters 5 > gpurun_out/r3s/pmc.txt 2>&1 || exit 3
bash tools/pmc_one.sh dgrad_l3c2 python3 tools/conv_one.py --mode dgrad --shape 512,8,8,256,256,3,1,1 --iters 5 >> gpurun_out/r3s/pmc.txt 2>&1 || exit 3
bash tools/pmc_one.sh fwd_l1c3 python3 tools/conv_one.py --mode fwd --shape 512,32,32,64,256,1,1,0 --iters 5 >> gpurun_out/r3s/pmc.txt 2>&1 || exit 3
bash tools/pmc_one.sh w1_l3c1 python3 tools/conv_one.py --mode wgrad --shape 512,8,8,1024,256,1,1,0 --iters 5 >> gpurun_out/r3s/pmc.txt 2>&1 || exit 3
python tools/pmc_table.py gpurun_out/pmc > gpurun_out/r3s/pmc_table.txt 2>&1
for g in 0 1; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --per_gpu_batch 128 --graph $g > gpurun_out/r3s/b128_g$g.txt 2>&1 || exit 1
  timeout -k 10 200 python bench.py --steps 40 --warmup 10 --graph $g > gpurun_out/r3s/b256_g$g.txt 2>&1 || exit 1
done
