# Perf evidence: column-reduce unroll A/B (variant cr4 = round-2 loop), emulated 8-rank
# SyncBN cost on the step (fused xGMI exchange vs reduce/x·W/finalize vs none) at 256 and
# 128 images per GPU, per-shape conv table, step profile. Crash / timeout ends the script.
mkdir -p gpurun_out/r3s3
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > gpurun_out/r3s3/dist_tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
bash tools/gpu/ab_bench.sh 3 "base:" "cr4:SDX_EXT_VARIANT=cr4" > gpurun_out/r3s3/ab_cr.txt 2>&1 || exit 1
for pg in 256 128; do
  for kind in none fused emu; do
    if [ $kind = none ]; then e=""; else e="SDX_SYNCBN_EMU=8 SDX_SYNCBN_EMU_KIND=$kind"; fi
    env $e timeout -k 10 150 python bench.py --steps 40 --warmup 10 --per_gpu_batch $pg > gpurun_out/r3s3/emu_${pg}_${kind}.txt 2>&1 || exit 1
    echo "per_gpu $pg syncbn $kind: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3s3/emu_${pg}_${kind}.txt) $(grep 'host issue' gpurun_out/r3s3/emu_${pg}_${kind}.txt | head -1)" >> gpurun_out/r3s3/emu_summary.txt
  done
done
timeout -k 10 300 python tools/conv_bench.py --no_miopen --iters 30 > gpurun_out/r3s3/conv_bench.txt 2>&1 || exit 1
bash tools/profile_step.sh r3a > gpurun_out/r3s3/profile.txt 2>&1 || exit 1
# config-5 slice (SupCon, 224x224 ImageNet stem, LARS, 512 images/GPU): per-kernel summary
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc5 -o run -- python3 bench.py --config supcon224 --steps 4 --warmup 2 > gpurun_out/r3s3/cfg5_prof.log 2>&1 || exit 1
python tools/rocpd_to_csv.py /tmp/pc5 > /dev/null
d=$(dirname $(find /tmp/pc5 -name "run_kernel_trace.csv" | head -1))
python tools/rocprof_summary.py $d --steps 9 > gpurun_out/r3s3/cfg5_summary.txt
