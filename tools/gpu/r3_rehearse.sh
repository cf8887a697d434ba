# Rehearsal of the driver's N>1 bench launch on one GPU (2 and 4 ranks sharing cuda:0, gloo
# process group after RCCL refuses duplicated devices); the JSON line reports the SyncBN
# transport in use (xgmi-fused expected). Timing is meaningless (ranks share one GPU).
set -o pipefail
mkdir -p gpurun_out/r3r
cd "${GRAFT_REPO_ROOT:-.}"
NPROC=2 PORT=29571 bash tools/rehearse_multirank.sh > gpurun_out/r3r/np2.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
NPROC=4 PORT=29573 bash tools/rehearse_multirank.sh > gpurun_out/r3r/np4.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
