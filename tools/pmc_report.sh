#!/bin/bash
# rocprofv3 PMC counters for the hot kernels (conv fwd/dgrad/wgrad tiles, fused loss):
# MFMA busy / wave cycles, VALU and LDS instruction mix, LDS bank conflicts, L2 traffic.
# Counters are collected with --pmc only (no tracing domains), a few per pass.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc
mkdir -p $OUT
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
      "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
      "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
run() {   # name, command...
  local name=$1; shift
  local i=0
  for s in "${SETS[@]}"; do
    timeout -k 10 120 rocprofv3 --pmc $s --output-format csv -d $OUT/$name.$i -o run -- "$@" > /dev/null 2>&1
    i=$((i+1))
  done
}
run conv_fwd_l3c2 python3 tools/conv_one.py --mode fwd --shape 512,8,8,256,256,3,1,1 --iters 3
run conv_dgrad_l3c2 python3 tools/conv_one.py --mode dgrad --shape 512,8,8,256,256,3,1,1 --iters 3
run conv_wgrad_l3c2 python3 tools/conv_one.py --mode wgrad --shape 512,8,8,256,256,3,1,1 --iters 3
run conv_fwd_l1c3 python3 tools/conv_one.py --mode fwd --shape 512,32,32,64,256,1,1,0 --iters 3
run supcon_512 python3 tools/supcon_one.py --n 512 --iters 3
run supcon_8192 python3 tools/supcon_one.py --n 8192 --iters 3
python3 tools/pmc_table.py $OUT > $OUT/pmc_table.txt
cat $OUT/pmc_table.txt
