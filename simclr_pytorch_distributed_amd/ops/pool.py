"""Autograd binding of the NHWC pooling kernels (csrc/kernels/pool.hip): the ImageNet-stem
3x3/2 max-pool and the global average pool feeding the projection head."""
from __future__ import annotations

import torch

from . import _ext


class _MaxPool(torch.autograd.Function):
    """The forward records each window's first-max position (uint8, a quarter of the pooled
    input's bytes at 3x3/2); the backward scatters dy through it without re-reading the
    input (profiles/cfg5_supcon224_kernels_r3.txt: the recomputing kernel was 5.3 ms of a
    224x224 step)."""

    @staticmethod
    def forward(ctx, x, k, stride, pad):
        if not ctx.needs_input_grad[0]:
            return _ext.require().maxpool_fwd(x, k, stride, pad)
        y, idx = _ext.require().maxpool_fwd_idx(x, k, stride, pad)
        ctx.save_for_backward(idx)
        ctx.cfg = (x.shape[1], x.shape[2], k, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        return _ext.require().maxpool_bwd_idx(idx, dy.contiguous(), *ctx.cfg), None, None, None


class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return _ext.require().gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return _ext.require().gap_bwd(dy.float().contiguous(), *ctx.hw)


def maxpool_nhwc(x, k=3, stride=2, pad=1):
    return _MaxPool.apply(x, k, stride, pad)


def global_avgpool_nhwc(x):
    """NHWC bf16 [N,H,W,C] -> fp32 [N,C]."""
    return _GlobalAvgPool.apply(x)
