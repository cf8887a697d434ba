# BASELINE.json configs measurable on one GPU: headline (256/GPU), its 128/GPU slice
# (configs 3/4 per-GPU work), and config 5 (SupCon 224x224, LARS, 512 images/GPU).
# Writes gpurun_out/cfg/*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $O/b256.json 2> $O/b256.err || { tail -20 $O/b256.err; exit 1; }
tail -1 $O/b256.json
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --per_gpu_batch 128 > $O/b128.json 2> $O/b128.err || { tail -20 $O/b128.err; exit 1; }
tail -1 $O/b128.json
timeout -k 10 400 python bench.py --config supcon224 --steps ${CFG5_STEPS:-3} --warmup 1 > $O/cfg5.json 2> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
tail -1 $O/cfg5.json
grep -h "host issue" $O/*.err
