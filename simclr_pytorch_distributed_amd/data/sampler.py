"""Deterministic distributed sampling (replaces torch DistributedSampler,
main_supcon.py:195-199, 387).

Semantics preserved: each epoch a seeded permutation of the whole dataset
(seed + epoch), padded by wrapping to a multiple of the world size, rank ``r`` takes
every ``W``-th index starting at ``r``; batches of ``batch_size // W`` with the last
incomplete batch dropped (``drop_last=True``).

The permutation is produced on the host once per epoch with numpy (cheap), and
uploaded once; per-step index slices are views of that device tensor.
"""
from __future__ import annotations

import numpy as np
import torch


class DistributedIndexSampler:
    def __init__(self, n: int, batch_per_rank: int, world: int = 1, rank: int = 0, seed: int = 0,
                 shuffle: bool = True, drop_last: bool = True):
        self.n, self.b, self.world, self.rank = n, batch_per_rank, world, rank
        self.seed, self.shuffle, self.drop_last = seed, shuffle, drop_last
        self.epoch = 0
        self.num_samples = (n + world - 1) // world
        self.total = self.num_samples * world

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self) -> np.ndarray:
        if self.shuffle:
            g = np.random.default_rng(self.seed + self.epoch)
            idx = g.permutation(self.n)
        else:
            idx = np.arange(self.n)
        pad = self.total - self.n
        if pad > 0:
            idx = np.concatenate([idx, idx[:pad]])
        return idx[self.rank:self.total:self.world]

    def __len__(self):
        if self.drop_last:
            return self.num_samples // self.b
        return (self.num_samples + self.b - 1) // self.b

    def batches(self, device=None):
        idx = torch.from_numpy(self.indices().astype(np.int64))
        if device is not None:
            idx = idx.to(device, non_blocking=True)
        for i in range(len(self)):
            yield idx[i * self.b:(i + 1) * self.b]
