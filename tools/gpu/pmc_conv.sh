# PMC passes (one rocprofv3 --pmc run per counter set) over tools/conv_one.py for one conv:
#   bash tools/gpu/pmc_conv.sh NAME MODE SHAPE CFG   -> gpurun_out/pmc2/NAME.<i>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
NAME=$1; MODE=$2; SHAPE=$3; CFG=$4
OUT=gpurun_out/pmc2; mkdir -p $OUT
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
      "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL"
      "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
      "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
      "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS")
i=0
for s in "${SETS[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $s --output-format csv -d $OUT/$NAME.$i -o run -- python3 tools/conv_one.py --mode $MODE --shape $SHAPE --cfg $CFG --iters 10 > /dev/null 2>&1 || echo "set $i failed"
  i=$((i+1))
done
