# ResNet-50 W=2 vs W=1 with the fwd/dgrad tile config pinned (identical per-tile statistic partials)
mkdir -p gpurun_out/diag
d() { timeout -k 10 300 python -u tools/dist_diag.py "$@" >> gpurun_out/diag/dist_diag4.txt 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc" >> gpurun_out/diag/dist_diag4.txt; exit $rc; }; }
d resnet50 xgmi "SDX_CONV_CFG=4" "SDX_CONV_CFG=4"
d resnet50 "" "SDX_CONV_CFG=4" "SDX_CONV_CFG=4"
d resnet50 xgmi "SDX_CONV_CFG=0" "SDX_CONV_CFG=0"
d resnet18 xgmi "SDX_CONV_CFG=4" "SDX_CONV_CFG=4"
