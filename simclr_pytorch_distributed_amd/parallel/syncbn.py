"""Cross-replica BatchNorm for the torch (stock-op) backend — works on gloo/CPU and RCCL.

The native gfx950 path does SyncBN inside ops/bn.py (one fp64 all-reduce of the
epilogue-produced Σy/Σy² per layer). This module provides the same semantics for the
torch backend (CPU runs, oracle), replacing ``torch.nn.SyncBatchNorm`` (CUDA-only,
reference main_supcon.py:222-224): local [Σx, Σx²] are summed across ranks with a
differentiable all-reduce (backward = all-reduce of the statistic gradients), so the
normalisation and its gradient equal full-global-batch BatchNorm.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn


class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        y = x.clone()
        dist.all_reduce(y, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        dist.all_reduce(g, group=ctx.group)
        return g, None


def all_reduce_sum_grad(x, group=None):
    return _AllReduceSum.apply(x, group)


class SyncBatchNorm2d(nn.BatchNorm2d):
    """BatchNorm2d whose training statistics are global over a process group."""

    def __init__(self, *a, group=None, **kw):
        super().__init__(*a, **kw)
        self.group = group

    def forward(self, x):
        if not self.training or not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return super().forward(x)
        C = x.shape[1]
        xf = x.float()
        n_local = x.numel() // C
        s1 = xf.sum(dim=(0, 2, 3))
        s2 = (xf * xf).sum(dim=(0, 2, 3))
        cnt = torch.tensor([float(n_local)], device=x.device, dtype=torch.float32)
        stats = all_reduce_sum_grad(torch.cat([s1, s2, cnt]), self.group)
        n = stats[-1]
        mean = stats[:C] / n
        var = stats[C:2 * C] / n - mean * mean
        with torch.no_grad():
            if self.track_running_stats:
                m = self.momentum if self.momentum is not None else 0.1
                unbiased = var.detach() * n / (n - 1)
                self.running_mean.mul_(1 - m).add_(m * mean.detach())
                self.running_var.mul_(1 - m).add_(m * unbiased)
                self.num_batches_tracked.add_(1)
        inv = torch.rsqrt(var + self.eps)
        y = (xf - mean.view(1, C, 1, 1)) * inv.view(1, C, 1, 1)
        if self.affine:
            y = y * self.weight.view(1, C, 1, 1) + self.bias.view(1, C, 1, 1)
        return y.to(x.dtype)


def convert_sync_bn(module: nn.Module, group=None) -> nn.Module:
    out = module
    if isinstance(module, nn.BatchNorm2d) and not isinstance(module, SyncBatchNorm2d):
        out = SyncBatchNorm2d(module.num_features, module.eps, module.momentum, module.affine,
                              module.track_running_stats, group=group)
        if module.affine:
            with torch.no_grad():
                out.weight.copy_(module.weight)
                out.bias.copy_(module.bias)
        out.running_mean = module.running_mean
        out.running_var = module.running_var
        out.num_batches_tracked = module.num_batches_tracked
    for name, child in module.named_children():
        out.add_module(name, convert_sync_bn(child, group))
    return out
