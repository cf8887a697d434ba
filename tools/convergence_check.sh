#!/bin/bash
# Short SimCLR pretraining on synthetic CIFAR-shaped data with the native gfx950 path and
# the torch (MIOpen/hipBLASLt) path from the same seed, then a linear probe on the
# native checkpoint. Loss curves / accuracies land in $OUT/*.log.
set -e
OUT=${OUT:-gpurun_out/conv_check}
EPOCHS=${EPOCHS:-6}
mkdir -p $OUT
COMMON="--ngpu 1 --batch_size 256 --learning_rate 0.5 --temp 0.5 --cosine --method SimCLR --synthetic \
  --synthetic_size 10240 --epochs $EPOCHS --print_freq 10 --save_freq 1000 --seed 1"
timeout -k 10 400 python main_supcon.py $COMMON --backend native --work_dir $OUT/native > $OUT/native.log 2>&1
timeout -k 10 400 python main_supcon.py $COMMON --backend torch --work_dir $OUT/torch > $OUT/torch.log 2>&1
CKPT=$(ls -t $(find $OUT/native -name last.pth) | head -1)
timeout -k 10 400 python main_linear.py --synthetic --seed 1 --synthetic_size 10240 --epochs 10 --batch_size 256 \
  --learning_rate 5 --ckpt $CKPT --work_dir $OUT/linear --print_freq 20 > $OUT/linear.log 2>&1
