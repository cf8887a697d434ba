# Ablation timing of one conv shape across SDX_IGEMM_ABLATE bits and tile configs:
#   bash tools/gpu/ablate_conv.sh MODE SHAPE "CFGS" "BITS"  -> stdout table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
MODE=$1; SHAPE=$2; CFGS=${3:-"4 6"}; BITS=${4:-"0 4 2 6 8 12"}
for c in $CFGS; do for b in $BITS; do
  r=$(SDX_IGEMM_ABLATE=$b timeout -k 10 60 python tools/conv_one.py --mode $MODE --shape $SHAPE --cfg $c --iters 50 2>/dev/null | tail -1) || exit 1
  echo "cfg $c ablate $b: $r"
done; done
