"""Autograd binding of the fused BatchNorm kernels (csrc/kernels/bn.hip), with SyncBN.

``bn_act(y, sums, bn, relu)`` and ``bn_add_act(y, sums, bn, res=..., ...)`` apply a
training-mode BatchNorm whose statistics ``sums`` (fp64 [2, C] Σy, Σy²) were produced by
the convolution epilogue. With a process group (SyncBN, reference main_supcon.py:222-224)
the forward all-reduces those 2C doubles and the backward all-reduces the [k, C]
gradient sums — one small RCCL all-reduce per BN per direction (the stock SyncBN does an
all-gather of mean/invstd/count instead).

Residual forms (networks/resnet_big.py:57-67): ``relu(bn3(y3) + bn_s(ys))`` for a
projection shortcut and ``relu(bn3(y3) + x)`` for the identity shortcut, each one
elementwise pass forward and one reduce + one elementwise pass backward.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import _ext
from ..parallel import comm


def _allreduce(t: torch.Tensor, group):
    if group is not None:
        dist.all_reduce(t, group=group)
    return t


def _world(group) -> int:
    return comm.group_size(group)


def _gscale(group) -> float:
    """dγ/dβ factor: the backward sums are all-reduced (global), but the parameter
    gradient must stay this rank's share — torch SyncBatchNorm returns the local
    grad_weight/grad_bias, which the DDP mean turns into global / W."""
    return 1.0 / _world(group)


def _finalize(m, sums, bn, count, training, group):
    if training:
        _allreduce(sums, group)
        sc, sh, mean, inv = m.bn_finalize(sums, float(count), bn.weight.detach(), bn.bias.detach(), bn.eps,
                                          bn.momentum if bn.momentum is not None else 0.1, bn.track_running_stats,
                                          bn.running_mean, bn.running_var)
        if bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
        return sc, sh, mean, inv
    sc, sh = m.bn_eval_affine(bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var, bn.eps)
    return sc, sh, None, None


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, sums, gamma, beta, bn, relu, training, group):
        m = _ext.require()
        C = y.shape[-1]
        count = (y.numel() // C) * _world(group)
        sc, sh, mean, inv = _finalize(m, sums, bn, count, training, group)
        out = m.bn_apply(y, sc, sh, None, None, None, 0, relu)
        if training:
            ctx.save_for_backward(y, out if relu else None, gamma, mean, inv)
        ctx.relu, ctx.count, ctx.group = relu, count, group
        return out

    @staticmethod
    def backward(ctx, dout):
        m = _ext.require()
        y, out, gamma, mean, inv = ctx.saved_tensors
        dout = dout.contiguous()
        s = m.bn_bwd_reduce(dout, out, y, mean, None, None)
        _allreduce(s, ctx.group)
        ca, _, dga, dba, _, _ = m.bn_bwd_coef(s, float(ctx.count), gamma.detach(), mean, inv, None, None, None,
                                              grad_scale=_gscale(ctx.group))
        dy, _, _ = m.bn_bwd_apply(dout, out, y, ca, None, None, False)
        return dy, None, dga, dba, None, None, None, None


class _BNAddAct(torch.autograd.Function):
    """relu(bn_a(ya) + bn_b(yb)) [projection] or relu(bn_a(ya) + x) [identity]."""

    @staticmethod
    def forward(ctx, ya, sa, ga, ba, yb, sb, gb, bb, x, bn_a, bn_b, training, group):
        m = _ext.require()
        C = ya.shape[-1]
        count = (ya.numel() // C) * _world(group)
        sca, sha, mean_a, inv_a = _finalize(m, sa, bn_a, count, training, group)
        if yb is not None:
            scb, shb, mean_b, inv_b = _finalize(m, sb, bn_b, count, training, group)
            out = m.bn_apply(ya, sca, sha, yb, scb, shb, 1, True)
        else:
            mean_b = inv_b = None
            out = m.bn_apply(ya, sca, sha, x, None, None, 2, True)
        if training:
            ctx.save_for_backward(ya, yb, out, ga, gb, mean_a, inv_a, mean_b, inv_b)
        ctx.count, ctx.group, ctx.proj = count, group, yb is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        m = _ext.require()
        ya, yb, out, ga, gb, mean_a, inv_a, mean_b, inv_b = ctx.saved_tensors
        dout = dout.contiguous()
        if ctx.proj:
            s = m.bn_bwd_reduce(dout, out, ya, mean_a, yb, mean_b)
            _allreduce(s, ctx.group)
            ca, cb, dga, dba, dgb, dbb = m.bn_bwd_coef(s, float(ctx.count), ga.detach(), mean_a, inv_a,
                                                       gb.detach(), mean_b, inv_b, grad_scale=_gscale(ctx.group))
            dya, dyb, _ = m.bn_bwd_apply(dout, out, ya, ca, yb, cb, False)
            return dya, None, dga, dba, dyb, None, dgb, dbb, None, None, None, None, None
        s = m.bn_bwd_reduce(dout, out, ya, mean_a, None, None)
        _allreduce(s, ctx.group)
        ca, _, dga, dba, _, _ = m.bn_bwd_coef(s, float(ctx.count), ga.detach(), mean_a, inv_a, None, None, None,
                                              grad_scale=_gscale(ctx.group))
        dya, _, dz = m.bn_bwd_apply(dout, out, ya, ca, None, None, True)
        return dya, None, dga, dba, None, None, None, None, dz, None, None, None, None


def bn_act(y, sums, bn, relu: bool = True, training: bool = True, group=None):
    return _BNAct.apply(y, sums, bn.weight, bn.bias, bn, relu, training, group)


def bn_add_act(ya, sa, bn_a, yb=None, sb=None, bn_b=None, x: Optional[torch.Tensor] = None,
               training: bool = True, group=None):
    gb = bn_b.weight if bn_b is not None else None
    bb = bn_b.bias if bn_b is not None else None
    return _BNAddAct.apply(ya, sa, bn_a.weight, bn_a.bias, yb, sb, gb, bb, x, bn_a, bn_b, training, group)
