set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp9; mkdir -p $O
for b in 0 2 8 10 4 6 14; do
  echo "== abl ablate $b"
  SDX_EXT_VARIANT=abl SDX_IGEMM_ABLATE=$b timeout -k 10 60 python tools/igemm_trace.py --cfg 6 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
  SDX_EXT_VARIANT=abl SDX_IGEMM_ABLATE=$b timeout -k 10 60 python tools/conv_one.py --mode fwd --shape 512,8,8,256,256,3,1,1 --cfg 6 --iters 50 2>&1 | tail -1
done > $O/abl.txt 2>&1
for v in noprio nosgb ""; do
  echo "== variant '$v'"
  SDX_EXT_VARIANT=$v timeout -k 10 60 python tools/igemm_trace.py --cfg 6 2>&1 | grep -v amdgpu.ids | head -6 || exit 1
  SDX_EXT_VARIANT=$v timeout -k 10 60 python tools/conv_one.py --mode fwd --shape 512,8,8,256,256,3,1,1 --cfg 6 --iters 50 2>&1 | tail -1
done > $O/var.txt 2>&1
cat $O/abl.txt $O/var.txt
