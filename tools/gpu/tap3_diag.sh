#!/bin/bash
# Tap-reuse loop diagnosis: in-kernel timelines (SDX_IGEMM_TRACE) and ablations (the abl
# variant build: csrc/build.py --variant abl --define SDX_W1_ABL=1) of l1 / l3 3x3 fwd,
# tap cfgs vs the implicit-GEMM configs auto picks. -> gpurun_out/tap3diag/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/tap3diag
mkdir -p $O
L3=512,8,8,256,256,3,1,1
L2=512,16,16,128,128,3,1,1
L1=512,32,32,64,64,3,1,1
{
for spec in "$L3 12" "$L3 6" "$L3 13" "$L1 11" "$L1 1" "$L2 12" "$L2 13" "$L2 4"; do
  set -- $spec
  echo "== trace fwd $1 cfg $2"
  timeout -k 10 60 python tools/igemm_trace.py --mode fwd --shape $1 --cfg $2 2>&1 | grep -v amdgpu.ids || exit 1
done
} > $O/trace.txt 2>&1 || { tail -20 $O/trace.txt; exit 1; }
{
for spec in "$L3 12" "$L3 6" "$L1 11" "$L2 12"; do
  set -- $spec
  for b in 0 2 4 6 8 12 14; do
    r=$(SDX_EXT_VARIANT=abl SDX_IGEMM_ABLATE=$b timeout -k 10 60 python tools/conv_one.py --mode fwd --shape $1 --cfg $2 --iters 50 2>/dev/null | tail -1) || exit 1
    echo "$1 cfg $2 ablate $b: $r"
  done
done
} > $O/ablate.txt 2>&1 || { tail -20 $O/ablate.txt; exit 1; }
cat $O/ablate.txt
grep -E "==|wave|K-tiles" $O/trace.txt
