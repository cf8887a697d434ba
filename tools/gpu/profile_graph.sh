# Kernel trace of the hipGraph-replayed step (bench.py --graph 1) -> gpurun_out/prof_graph/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/prof_graph
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pg -o run -- python3 bench.py --steps 10 --warmup 3 --graph 1 > /tmp/pg.log 2>&1 || { tail -20 /tmp/pg.log; exit 1; }
python tools/rocpd_to_csv.py /tmp/pg > /dev/null
d=$(dirname $(find /tmp/pg -name "run_kernel_trace.csv" | head -1))
python tools/rocprof_summary.py $d --steps 8 > $O/summary.txt
python tools/step_timeline.py $d --dump $O/step_kernels.txt > $O/timeline.txt
head -12 $O/timeline.txt; tail -4 $O/timeline.txt
