#!/bin/bash
# HIP API call statistics of the bench step (where the host issue time goes): rocprofv3
# --hip-trace --stats (no counters) -> gpurun_out/hostapi/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/hostapi
mkdir -p $O
timeout -k 10 240 rocprofv3 --hip-trace --stats --output-format csv -d /tmp/ha -o run -- python3 bench.py --steps 20 --warmup 5 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
find /tmp/ha -name "*stats.csv" -exec cp {} $O/ \;
ls $O
head -25 $O/*hip_api_stats.csv
