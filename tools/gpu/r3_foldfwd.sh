# Forward half of the BN3 fold: fold tests (parity, SyncBN emulation, engine), then the bench
# A/B against SDX_BN3_FOLD_FWD=0 and a step profile. A crash / timeout ends the script.
set -o pipefail
mkdir -p gpurun_out/r3ff
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_comm.py tests/test_gpu_misc.py -v -k "fold or syncbn_path or engine or stage" --timeout 300 --timeout-method thread > gpurun_out/r3ff/tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
bash tools/gpu/ab_bench.sh 3 "ff:" "nf:SDX_BN3_FOLD_FWD=0" > gpurun_out/r3ff/ab.txt 2>&1 || exit 1
bash tools/profile_step.sh r3ff > gpurun_out/r3ff/profile.txt 2>&1 || exit 1
