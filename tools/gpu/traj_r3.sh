# Teacher-forced + free-running R50 trajectory probes; outputs under gpurun_out/tf
set -o pipefail
mkdir -p gpurun_out/tf
timeout -k 10 300 python -u tools/trajectory_tf.py tf resnet50 30 0.05 128 > gpurun_out/tf/tf_r50_lr05.txt 2>&1 &&
timeout -k 10 240 python -u tools/trajectory_tf.py free resnet50 30 0.05 128 > gpurun_out/tf/free_r50_lr05.txt 2>&1 &&
timeout -k 10 240 python -u tools/trajectory_tf.py free resnet50 30 0.02 128 > gpurun_out/tf/free_r50_lr02.txt 2>&1 &&
SDX_BN3_FOLD=0 timeout -k 10 300 python -u tools/trajectory_tf.py tf resnet50 30 0.05 128 > gpurun_out/tf/tf_r50_lr05_nofold.txt 2>&1
