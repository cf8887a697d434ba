set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pp17; mkdir -p $O
for v in "SDX_DGRAD_MERGE=0 SDX_CONV_D6=0" "SDX_DGRAD_MERGE=0" "SDX_CONV_D6=0" "SDX_SPLITK_MERGE=0" "X=1"; do
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -s -k "trajectory_tracks" > $O/t.log 2>&1; rc=$?
  echo "$v rc=$rc $(grep 'window means' $O/t.log)"
done
