# ResNet-50 W=2 vs W=1 step difference: which path carries it (fold, dgrad statistics hand-off, transport)
mkdir -p gpurun_out/diag
d() { timeout -k 10 300 python -u tools/dist_diag.py "$@" >> gpurun_out/diag/dist_diag.txt 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc" >> gpurun_out/diag/dist_diag.txt; exit $rc; }; }
d resnet18 xgmi "" ""
d resnet50 xgmi "" ""
d resnet50 "" "" ""
d resnet50 xgmi "SDX_BN3_FOLD=0" "SDX_BN3_FOLD=0"
d resnet50 xgmi "" "SDX_BN3_FOLD=0"
d resnet50 xgmi "SDX_DGRAD_BNSTAT=0 SDX_BN3_FOLD=0" "SDX_DGRAD_BNSTAT=0 SDX_BN3_FOLD=0"
d resnet50 xgmi "SDX_FUSED_HEAD=0" "SDX_FUSED_HEAD=0"
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -q -x --timeout 200 --timeout-method thread > gpurun_out/diag/comm_tests.txt 2>&1
