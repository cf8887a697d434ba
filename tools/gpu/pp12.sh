set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp12; mkdir -p $O
timeout -k 10 300 python tools/syncbn_latency.py 2,4,8 200 > $O/syncbn_latency.txt 2>&1 || { tail -20 $O/syncbn_latency.txt; exit 1; }
grep -A4 summary $O/syncbn_latency.txt
for mode in none emu fused solo; do
  case $mode in
    none) E="";;
    emu) E="SDX_SYNCBN_EMU=8 SDX_SYNCBN_EMU_KIND=emu";;
    fused) E="SDX_SYNCBN_EMU=8 SDX_SYNCBN_EMU_KIND=fused";;
    solo) E="SDX_SYNCBN_EMU=8 SDX_SYNCBN_EMU_KIND=fused SDX_SYNCBN_EMU_SOLO=1";;
  esac
  env $E timeout -k 10 200 python bench.py --per_gpu_batch 128 --steps 30 > $O/b128_$mode.log 2>&1 || { tail -5 $O/b128_$mode.log; exit 1; }
  echo "$mode $(grep -o '"ms_per_step": [0-9.]*' $O/b128_$mode.log)"
done
