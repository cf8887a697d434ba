set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pp13; mkdir -p $O
for mode in none solo emu; do
  case $mode in
    none) E="";;
    emu) E="SDX_SYNCBN_EMU=8 SDX_SYNCBN_EMU_KIND=emu";;
    solo) E="SDX_SYNCBN_EMU=8 SDX_SYNCBN_EMU_KIND=fused SDX_SYNCBN_EMU_SOLO=1";;
  esac
  rm -rf /tmp/pp_$mode
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pp_$mode -o run -- python3 bench.py --per_gpu_batch 128 --steps 10 --warmup 3 > $O/log_$mode.txt 2>&1 || { tail -20 $O/log_$mode.txt; exit 1; }
  python tools/rocpd_to_csv.py /tmp/pp_$mode > /dev/null
  d=$(dirname $(find /tmp/pp_$mode -name "run_kernel_trace.csv" | head -1))
  python tools/rocprof_summary.py $d --steps 16 > $O/summary_$mode.txt
  head -3 $O/summary_$mode.txt
done
