# Host issue cost of the native step (per-phase host time, idle and full queue; cProfile of
# 20 steps) and the device duration of every SyncBN-latency kernel (rocprofv3 kernel trace of
# tools/syncbn_latency.py). A crash / timeout ends the script.
mkdir -p gpurun_out/r3h
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 python -u tools/host_phases.py > gpurun_out/r3h/phases.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/host_profile.py > gpurun_out/r3h/cprofile.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/lat -o run -- python3 tools/syncbn_latency.py 8 200 > gpurun_out/r3h/lat.txt 2>&1 || exit $?
python tools/rocpd_to_csv.py /tmp/lat > /dev/null
d=$(dirname $(find /tmp/lat -name "run_kernel_trace.csv" | head -1))
python tools/kernel_durations.py $d > gpurun_out/r3h/lat_kernels.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3h/gpu_tests.txt 2>&1; rc=$?; [ $rc -le 1 ] || exit $rc
