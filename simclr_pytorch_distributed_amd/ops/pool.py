"""Autograd binding of the NHWC pooling kernels (csrc/kernels/pool.hip): the ImageNet-stem
3x3/2 max-pool and the global average pool feeding the projection head."""
from __future__ import annotations

import torch

from . import _ext


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad):
        y = _ext.require().maxpool_fwd(x, k, stride, pad)
        ctx.save_for_backward(x, y)
        ctx.cfg = (k, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        return _ext.require().maxpool_bwd(x, y, dy.contiguous(), *ctx.cfg), None, None, None


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
