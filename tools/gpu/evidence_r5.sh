#!/bin/bash
# Round-5 kernel evidence: per-shape conv table (tools/conv_bench.py vs MIOpen) and PMC passes
# of the tap-reuse 3x3 loop on l3.x.c2 (cfg 12) and l1.x.c2 (cfg 11), fwd and dgrad.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ev5
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/ev5/conv_bench.txt 2>&1 || { tail -20 gpurun_out/ev5/conv_bench.txt; exit 1; }
tail -8 gpurun_out/ev5/conv_bench.txt
rm -rf gpurun_out/pmc2
bash tools/gpu/pmc_conv.sh fwd_l3c2_tap fwd 512,8,8,256,256,3,1,1 12
bash tools/gpu/pmc_conv.sh dgrad_l3c2_tap dgrad 512,8,8,256,256,3,1,1 12
bash tools/gpu/pmc_conv.sh fwd_l1c2_tap fwd 512,32,32,64,64,3,1,1 11
python tools/pmc_table.py gpurun_out/pmc2 > gpurun_out/ev5/pmc.txt 2>&1
cat gpurun_out/ev5/pmc.txt | cut -c1-200
