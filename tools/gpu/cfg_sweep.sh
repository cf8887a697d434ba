#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
timeout -k 10 600 python tools/cfg_sweep.py > gpurun_out/sweep/cfg_sweep.txt 2>&1 || { tail -20 gpurun_out/sweep/cfg_sweep.txt; exit 1; }
grep -v amdgpu gpurun_out/sweep/cfg_sweep.txt
hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_ab tools/mfma_ab/mfma_ab.hip && timeout -k 10 120 /tmp/mfma_ab > gpurun_out/sweep/mfma_ab.txt 2>&1 || { tail -5 gpurun_out/sweep/mfma_ab.txt; exit 1; }
cat gpurun_out/sweep/mfma_ab.txt
