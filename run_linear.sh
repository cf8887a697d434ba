#!/bin/bash
# README recipe (reference run_linear.sh): linear probe, lr 5, batch 256, 1 GPU.
export PYTHONPATH=.
python main_linear.py \
    --learning_rate 5 \
    --batch_size 256 \
    --ckpt ${CKPT:-path/to/ckpt} "$@"
