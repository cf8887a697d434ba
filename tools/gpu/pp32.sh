#!/bin/bash
# end-state rehearsal of the driver's N>1 bench launch at 2 and 4 ranks on one GPU
cd "${GRAFT_REPO_ROOT:-.}"
NPROC=2 PORT=29561 timeout -k 10 600 bash tools/rehearse_multirank.sh || exit 1
NPROC=4 PORT=29571 timeout -k 10 600 bash tools/rehearse_multirank.sh || exit 1
