# fused SyncBN exchange + native linear-probe + supcon tests, latency table, supcon PMC at
# N = 8192, the multi-rank tests, then the R50 trajectory sweep. A crash / timeout of a GPU
# step ends the script (exit codes other than 0 = pass, 1 = test failures).
mkdir -p gpurun_out/r3s2
run() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/r3s2/$name.txt 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r3s2/status.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run unit_tests 500 python -u -m pytest tests/test_gpu_xgmi.py tests/test_gpu_comm.py tests/test_gpu_probe.py tests/test_gpu_supcon.py -v --timeout 200 --timeout-method thread
run latency 120 python -u tools/syncbn_latency.py 8 200
run supcon_time 120 python -u tools/supcon_one.py --n 8192 --iters 20
bash tools/pmc_one.sh supcon_8192 python3 tools/supcon_one.py --n 8192 --iters 3 > gpurun_out/r3s2/pmc.txt 2>&1 || exit 3
python tools/pmc_table.py gpurun_out/pmc > gpurun_out/r3s2/pmc_table.txt 2>&1
run dist_tests 700 python -u -m pytest tests/test_gpu_dist.py -v --timeout 600 --timeout-method thread
bash tools/gpu/traj_r3b.sh
