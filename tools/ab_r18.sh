set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r18
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_misc.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k imagenet > $O/t5.log 2>&1 || { tail -30 $O/t5.log; exit 1; }
tail -1 $O/t5.log
for c in 5 0; do
  timeout -k 10 200 python tools/conv_bench.py --no_miopen --cfg $c > $O/cb_cfg$c.txt 2>&1 || exit 1
  SDX_IGEMM_RING=1 timeout -k 10 200 python tools/conv_bench.py --no_miopen --cfg $c > $O/cb_cfg${c}_ring.txt 2>&1 || exit 1
done
for f in $O/cb_*.txt; do echo $f; grep TOTAL $f | head -2; done
