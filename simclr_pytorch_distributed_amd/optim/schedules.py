"""Learning-rate schedules, value-identical to the reference (util.py:54-76).

* :func:`adjust_learning_rate` — per-epoch, 1-indexed: cosine annealing
  to ``eta_min = lr * decay_rate**3`` or multi-step decay.
* :func:`warmup_learning_rate` — per-iteration linear warm-up from ``warmup_from`` to
  ``warmup_to`` across ``warm_epochs`` epochs.

Both return the lr they set so the engine can keep it on device for the fused
optimizer without a host round-trip.
"""
from __future__ import annotations

import math


def lr_at_epoch(args, epoch: int) -> float:
    lr = args.learning_rate
    if args.cosine:
        eta_min = lr * (args.lr_decay_rate ** 3)
        lr = eta_min + (lr - eta_min) * (1 + math.cos(math.pi * epoch / args.epochs)) / 2
    else:
        steps = sum(1 for e in args.lr_decay_epochs if epoch > e)
        if steps > 0:
            lr = lr * (args.lr_decay_rate ** steps)
    return lr


def set_lr(optimizer, lr: float):
    for group in optimizer.param_groups:
        group["lr"] = lr


def adjust_learning_rate(args, optimizer, epoch: int) -> float:
    lr = lr_at_epoch(args, epoch)
    set_lr(optimizer, lr)
    return lr


def warmup_lr(args, epoch: int, batch_id: int, total_batches: int):
    if getattr(args, "warm", False) and epoch <= args.warm_epochs:
        p = (batch_id + (epoch - 1) * total_batches) / (args.warm_epochs * total_batches)
        return args.warmup_from + p * (args.warmup_to - args.warmup_from)
    return None


def warmup_learning_rate(args, epoch: int, batch_id: int, total_batches: int, optimizer):
    lr = warmup_lr(args, epoch, batch_id, total_batches)
    if lr is not None:
        set_lr(optimizer, lr)
    return lr
