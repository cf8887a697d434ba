#!/bin/bash
# PMC counter passes (the pmc_report.sh sets, one rocprofv3 --pmc run each) for ONE command:
#   bash tools/pmc_one.sh <name> <command...>   -> gpurun_out/pmc/<name>.<set>/ + pmc_table row
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc
mkdir -p $OUT
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
      "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
      "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
name=$1; shift
i=0
for s in "${SETS[@]}"; do
  timeout -k 10 120 rocprofv3 --pmc $s --output-format csv -d $OUT/$name.$i -o run -- "$@" > /dev/null 2>&1
  i=$((i+1))
done
