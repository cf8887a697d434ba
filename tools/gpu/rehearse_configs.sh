#!/bin/bash
# The driver's multi-GPU bench commands rehearsed on ONE GPU: BASELINE
# config 4 at W=8 (cifar100, global batch 1024 = 128 per rank) and config 3 at W=2 (global
# batch 256), each through torch.distributed.run exactly as the driver launches it; RCCL
# refuses several ranks on one device, so the rehearsal falls back to the gloo process group.
# -> gpurun_out/multirank/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
NPROC=8 TAG=_cfg4 TLIM=600 PORT=29571 BENCH_ARGS="--dataset cifar100 --global_batch 1024" bash tools/rehearse_multirank.sh || exit $?
NPROC=2 TAG=_cfg3 TLIM=300 PORT=29581 BENCH_ARGS="--global_batch 256" bash tools/rehearse_multirank.sh
