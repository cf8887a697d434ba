# Rehearse the driver's N>1 bench launch (torch.distributed.run, one rank per "GPU") on a
# 1-GPU box: both ranks share cuda:0 (comm.init_distributed maps local ranks round-robin).
# First the production path (RCCL process group + RCCL SyncBN communicator); if RCCL
# refuses two ranks on one device (plain error, exit 1), the gloo process group instead.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
# NPROC (default 2): ranks to start (<= 16 on one box); PORT: rendezvous port; BENCH_ARGS:
# extra bench.py arguments (e.g. "--dataset cifar100 --global_batch 1024", BASELINE config 4);
# TAG: log-name suffix; TLIM: per-launch time limit in seconds
NP=${NPROC:-2}
PORT=${PORT:-29561}
TLIM=${TLIM:-240}
SFX=${TAG:-}
O=gpurun_out/multirank
mkdir -p $O
run() {  # $1 = tag, rest = extra bench args
  tag=$1_np$NP$SFX; shift
  timeout -k 10 $TLIM python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
    --master-port $PORT bench.py --gpus $NP --steps 10 --warmup 3 $BENCH_ARGS "$@" > $O/$tag.log 2>&1
}
run nccl; rc=$?
echo "nccl rc=$rc"; grep '"metric"' $O/nccl_np$NP$SFX.log || tail -15 $O/nccl_np$NP$SFX.log
[ $rc -eq 0 ] && exit 0
[ $rc -ne 1 ] && exit $rc
run gloo --dist_backend gloo; rc=$?
echo "gloo rc=$rc"; grep '"metric"' $O/gloo_np$NP$SFX.log || tail -15 $O/gloo_np$NP$SFX.log
exit $rc
