# Round-end rehearsal: the whole GPU test tier, smoke(), the default bench.py run, then the
# supcon tile kernel time + PMC after the second LDS swizzle. A crash / timeout of a GPU
# step ends the script (exit codes other than 0 = pass, 1 = test failures).
mkdir -p gpurun_out/r3f
cd "${GRAFT_REPO_ROOT:-.}"
run() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/r3f/$name.txt 2>&1; local rc=$?; echo "$name rc=$rc" >> gpurun_out/r3f/status.txt; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 300 python -u bench.py
run supcon_time 120 python -u tools/supcon_one.py --n 8192 --iters 20
bash tools/pmc_one.sh supcon_8192 python3 tools/supcon_one.py --n 8192 --iters 3 > gpurun_out/r3f/pmc.txt 2>&1 || exit 3
python tools/pmc_table.py gpurun_out/pmc > gpurun_out/r3f/pmc_table.txt 2>&1
