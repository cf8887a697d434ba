# lr sweep of free-running R50 trajectories (native / fp32 / autocast / fp32 replica) and a longer teacher-forced run
set -o pipefail
mkdir -p gpurun_out/tf
timeout -k 10 300 python -u tools/trajectory_tf.py free resnet50 40 0.01 128 > gpurun_out/tf/free_r50_lr01.txt 2>&1 &&
timeout -k 10 300 python -u tools/trajectory_tf.py free resnet50 40 0.005 128 > gpurun_out/tf/free_r50_lr005.txt 2>&1 &&
timeout -k 10 300 python -u tools/trajectory_tf.py free resnet50 40 0.02 128 > gpurun_out/tf/free_r50_lr02b.txt 2>&1 &&
timeout -k 10 300 python -u tools/trajectory_tf.py tf resnet50 40 0.01 128 > gpurun_out/tf/tf_r50_lr01.txt 2>&1
