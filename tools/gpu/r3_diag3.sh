# ResNet-50 W=2 vs W=1: bucket count / backend isolation
mkdir -p gpurun_out/diag
d() { timeout -k 10 300 python -u tools/dist_diag.py "$@" >> gpurun_out/diag/dist_diag3.txt 2>&1; local rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc" >> gpurun_out/diag/dist_diag3.txt; exit $rc; }; }
d resnet50 "" "" "SDX_BUCKET_MB=1000"
d resnet50 "" "SDX_TEST_BACKEND=torch" "SDX_TEST_BACKEND=torch"
d resnet18 "" "SDX_TEST_BACKEND=torch" "SDX_TEST_BACKEND=torch"
d resnet50 "" "SDX_WGRAD_STREAM=0" "SDX_WGRAD_STREAM=0"
