# chaos floor: two single-rank ResNet-50 / -18 steps that differ only in the BN-statistics summation order
mkdir -p gpurun_out/diag
d() { timeout -k 10 300 python -u tools/dist_diag.py "$@" >> gpurun_out/diag/dist_diag2.txt 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc" >> gpurun_out/diag/dist_diag2.txt; exit $rc; }; }
d resnet50 "" "" "SDX_STAT_FUSE=3" 1
d resnet18 "" "" "SDX_STAT_FUSE=3" 1
d resnet50 "" "" "SDX_BN3_FOLD=0" 1
