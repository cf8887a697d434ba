#!/bin/bash
# End-to-end pipeline on synthetic CIFAR-shaped data (no dataset downloads possible):
# SimCLR pretraining on the native gfx950 path -> checkpoint -> linear probe, plus the
# same probe on a randomly initialised encoder as the control.
set -e
# Note: on this synthetic data the pretrained features reach norms of ~10^3-10^4 (the collapse
# phase of SimCLR at lr 0.5 without warm-up, see profiles/convergence_r1.txt); the
# reference probe lr of 5 then diverges for ANY implementation, so the probe uses LIN_LR.
OUT=${OUT:-gpurun_out/e2e}
WORK=${WORK:-/tmp/sdx_e2e}
EPOCHS=${EPOCHS:-10}
LIN_LR=${LIN_LR:-0.05}
mkdir -p $OUT $WORK
timeout -k 10 600 python main_supcon.py --batch_size 256 --learning_rate 0.5 --temp 0.5 --cosine --method SimCLR \
  --synthetic --synthetic_size 50000 --epochs $EPOCHS --print_freq 50 --save_freq 1000 --seed 1 --backend native \
  --work_dir $WORK/pre > $OUT/pretrain.log 2>&1
CKPT=$(find $WORK/pre -name last.pth | head -1)
timeout -k 10 300 python main_linear.py --synthetic --seed 1 --synthetic_size 50000 --epochs 5 --batch_size 256 \
  --learning_rate $LIN_LR --ckpt $CKPT --work_dir $WORK/lin --print_freq 100 > $OUT/linear.log 2>&1
timeout -k 10 300 python main_linear.py --synthetic --seed 1 --synthetic_size 50000 --epochs 5 --batch_size 256 \
  --learning_rate $LIN_LR --work_dir $WORK/lin_rand --print_freq 100 > $OUT/linear_random.log 2>&1
grep -h "epoch .*total time" $OUT/pretrain.log | tail -3
grep -h "best accuracy" $OUT/linear.log $OUT/linear_random.log
