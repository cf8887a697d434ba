set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp3; mkdir -p $O
for v in "" ppearly; do
  echo "== variant '$v'"
  SDX_EXT_VARIANT=$v bash tools/gpu/ablate_conv.sh fwd 512,8,8,256,256,3,1,1 "6 5" "0 4 2 12" || exit 1
  SDX_EXT_VARIANT=$v bash tools/gpu/ablate_conv.sh fwd 512,16,16,128,128,3,1,1 "5" "0 4 2 12" || exit 1
  SDX_EXT_VARIANT=$v bash tools/gpu/ablate_conv.sh fwd 512,4,4,512,512,3,1,1 "5 6" "0" || exit 1
done > $O/ab.txt 2>&1
cat $O/ab.txt
