#!/bin/bash
# README recipe (reference run_supcon.sh): SimCLR, SyncBN, 100 epochs, lr 0.5, temp 0.5, cosine.
# One process per GPU over RCCL; set NGPU to the number of MI355X GPUs to use.
NGPU=${NGPU:-2}
export PYTHONPATH=.
python -m torch.distributed.run --nproc-per-node ${NGPU} --master-addr 127.0.0.1 --master-port 6015 main_supcon.py \
    --syncBN \
    --epochs 100 \
    --learning_rate 0.5 \
    --temp 0.5 \
    --cosine \
    --method SimCLR \
    --ngpu ${NGPU} "$@"
