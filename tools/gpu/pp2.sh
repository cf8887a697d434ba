set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp2; mkdir -p $O
bash tools/gpu/ablate_conv.sh fwd 512,8,8,256,256,3,1,1 "4 6 5" > $O/abl_l3c2.txt 2>&1 || exit 1
bash tools/gpu/ablate_conv.sh fwd 512,16,16,128,128,3,1,1 "4 6 5" > $O/abl_l2c2.txt 2>&1 || exit 1
cat $O/abl_l3c2.txt $O/abl_l2c2.txt
timeout -k 10 60 rocprofv3 --list-avail > $O/counters.txt 2>&1 || true
grep -o "TA_[A-Z_]*\|TD_[A-Z_]*\|TCP_[A-Z_]*" $O/counters.txt | sort -u | head -80 > $O/counters_short.txt || true
