set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r25
mkdir -p $O
for c in -1 0 1 2 3 4; do
  timeout -k 10 200 python tools/conv_bench.py --no_miopen --cfg $c > $O/cb_$c.txt 2>&1 || exit 1
done
for c in -1 0 1 2 3 4; do echo "== cfg $c"; grep -E "^l1\.(0|x)\.(c3|sc|c1) |^l2\.0\.c1 " $O/cb_$c.txt | grep -v wgrad | awk '{print $1,$2,$6}' | tr '\n' ';'; echo; done
