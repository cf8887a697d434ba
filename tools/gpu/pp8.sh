set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/pp8; mkdir -p $O
for c in 6 5; do timeout -k 10 60 python tools/igemm_trace.py --cfg $c > $O/trace_$c.txt 2>&1 || exit 1; done
timeout -k 10 60 python tools/igemm_trace.py --cfg 5 --shape 512,16,16,128,128,3,1,1 > $O/trace_5_l2.txt 2>&1 || exit 1
timeout -k 10 60 python tools/igemm_trace.py --cfg 4 --shape 512,16,16,128,128,3,1,1 > $O/trace_4_l2.txt 2>&1 || exit 1
cat $O/trace_6.txt $O/trace_5.txt $O/trace_5_l2.txt
