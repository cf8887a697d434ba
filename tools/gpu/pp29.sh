#!/bin/bash
# round-4 PMC: conv main loops (cfg 6 = DEPTH 6 256-wide tile, cfg 4 = round-3 128x128) on l3.x.c2 fwd/dgrad,
# the 1x1 / 3x3 / stride-2 3x3 wgrad kernels
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
C="python3 tools/conv_one.py --iters 10"
bash tools/pmc_one.sh fwd_l3c2_cfg6 $C --mode fwd --shape 512,8,8,256,256,3,1,1 --cfg 6 || exit 1
bash tools/pmc_one.sh dgrad_l3c2_cfg6 $C --mode dgrad --shape 512,8,8,256,256,3,1,1 --cfg 6 || exit 1
bash tools/pmc_one.sh fwd_l3c2_cfg4 $C --mode fwd --shape 512,8,8,256,256,3,1,1 --cfg 4 || exit 1
bash tools/pmc_one.sh w1_l3c1 $C --mode wgrad --shape 512,8,8,1024,256,1,1,0 || exit 1
bash tools/pmc_one.sh w3_l3c2 $C --mode wgrad --shape 512,8,8,256,256,3,1,1 || exit 1
bash tools/pmc_one.sh w3s2_l3c2 $C --mode wgrad --shape 512,16,16,256,256,3,2,1 || exit 1
python3 tools/pmc_table.py gpurun_out/pmc > gpurun_out/pmc/table_r4.txt
cat gpurun_out/pmc/table_r4.txt
