set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp5; mkdir -p $O
for b in 0 14 10 2; do
  echo "== cfg 6 ablate $b"
  SDX_IGEMM_ABLATE=$b timeout -k 10 60 python tools/igemm_trace.py --cfg 6 || exit 1
done > $O/trace.txt 2>&1
cat $O/trace.txt
