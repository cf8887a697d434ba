"""Fused ResNet building blocks: one autograd node per Bottleneck / BasicBlock / stem.

Forward and backward of a whole residual block are explicit kernel sequences (reference
math: networks/resnet_big.py:7-67), which lets the executor

* reuse one bf16 weight cache for all convs (one ``wprep`` launch per step);
* write every parameter gradient straight into its ``.grad`` sink (conv dW through the
  split-K reduce, BN dγ/dβ from the coefficient kernel) — no AccumulateGrad adds;
* fuse the residual-gradient sum into the last data-gradient GEMM epilogue
  (``dx = dgrad(conv1) + dgrad(shortcut) | + dz``) instead of a separate add pass;
* run SyncBN as one fp64 all-reduce per BN per direction;
* optionally (``SDX_FUSE_PROLOGUE=1``) never materialise the block-internal activations
  ``relu(bn1(y1))`` / ``relu(bn2(y2))``: the consuming conv applies BN+ReLU in its
  operand-load prologue (forward and weight gradient) and the BN backward recomputes the
  ReLU mask from ``y``. That saves one write + two reads per internal activation but
  forces register staging on those convs; with LDS-DMA staged convs the materialised
  path is faster, so it is the default.

Parameters are passed to ``apply`` only to keep the autograd graph connected (their
returned gradients are ``None``: the sinks already hold them); the bucket reducer is
notified through :mod:`ops.sinks`.
"""
from __future__ import annotations

import contextlib
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _ext, sinks
from ..parallel import comm
from .streams import SideWork

_STEM_SIDE = os.environ.get("SDX_STEM_SIDE", "0") == "1"


# off by default: with LDS-DMA staged convs, materialising relu(bn(y)) once is faster than
# the register-staged prologue conv (16.9 vs 17.3 ms/step, ResNet-50 bench)
FUSE_PROLOGUE = os.environ.get("SDX_FUSE_PROLOGUE", "0") == "1"


def _omask(like, training):
    """uint8 ReLU bitmask buffer (1 bit per element) for a block output, training only:
    BN backward reads it instead of the bf16 output."""
    if not training:
        return None
    return torch.empty(like.numel() // 8, dtype=torch.uint8, device=like.device)


def _world(group) -> int:
    return comm.group_size(group)


class _BN:
    """Per-BN forward state: finalize (train) or eval affine."""

    @staticmethod
    def forward(m, slab, bn, count, training, group):
        """``slab``: the conv epilogue's per-tile (Σy, Σy²). Single process: reduction +
        finalize in one launch; SyncBN: reduce, fp64 all-reduce, finalize."""
        if training:
            mom = bn.momentum if bn.momentum is not None else 0.1
            args = (float(count), bn.weight.detach(), bn.bias.detach(), bn.eps, mom, bn.track_running_stats,
                    bn.running_mean, bn.running_var)
            if group is None:
                return tuple(m.bn_stats_finalize(slab, *args))
            sums = m.bn_stats_reduce(slab)
            comm.small_all_reduce_(sums, group)
            sc, sh, mean, inv = m.bn_finalize(sums, *args)
            return sc, sh, mean, inv
        sc, sh = m.bn_eval_affine(bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var, bn.eps)
        return sc, sh, None, None


def _conv(m, x, w, stride, pad, stats, in_bn=None):
    """conv (+BN stat slab); ``in_bn=(scale, shift)``: x is a pre-BN tensor and the
    kernel feeds relu(x·scale + shift) to the GEMM."""
    isc, ish = in_bn if in_bn is not None else (None, None)
    y, slab = m.conv_fwd(x, w, stride, pad, stats, -1, isc, ish)
    return y, (slab if stats else None)


def _act(m, y, sc, sh):
    """Block-internal BN+ReLU: returns (tensor the next conv reads, its prologue affine)."""
    if FUSE_PROLOGUE:
        return y, (sc, sh)
    return m.bn_apply(y, sc, sh, None, None, None, 0, True), None


def _bn_bwd(m, dout, out, y, mean, inv, bn, count, group, y_b=None, mean_b=None, inv_b=None, bn_b=None,
            want_dz=False, mask=None):
    """BN(+second BN)+ReLU backward with dγ/dβ written into the parameter sinks.
    ReLU mask from ``out``, or (``out`` None) from ``mask=(scale, shift)``: y·scale+shift > 0."""
    msc, msh = mask if (out is None and mask is not None) else (None, None)
    snk = dict(sink_ga=sinks.target(bn.weight), sink_ba=sinks.target(bn.bias))
    if y_b is not None:
        snk.update(sink_gb=sinks.target(bn_b.weight), sink_bb=sinks.target(bn_b.bias))
    gb = bn_b.weight.detach() if y_b is not None else None
    if group is None:
        # elementwise reduce + (last-block) coefficients: two launches, no host round trip
        ca, cb, _, _, _, _ = m.bn_bwd_reduce_coef(dout, out, y, mean, y_b, mean_b, msc, msh, float(count),
                                                  bn.weight.detach(), inv, gb, inv_b, **snk)
    else:
        s = m.bn_bwd_reduce(dout, out, y, mean, y_b, mean_b, msc, msh)
        comm.small_all_reduce_(s, group)
        # dγ/dβ: this rank's share of the all-reduced sums (torch SyncBatchNorm + DDP mean)
        ca, cb, _, _, _, _ = m.bn_bwd_coef(s, float(count), bn.weight.detach(), mean, inv, gb, mean_b, inv_b, **snk,
                                           grad_scale=1.0 / _world(group))
    if y_b is None:
        dya, _, dz = m.bn_bwd_apply(dout, out, y, ca, None, None, want_dz, msc, msh)
        return dya, None, dz
    dya, dyb, _ = m.bn_bwd_apply(dout, out, y, ca, y_b, cb, False)
    return dya, dyb, None


def _wgrad(m, dy, x, cv, stride, pad, in_bn=None):
    """Weight gradient into the parameter sink, on the side stream (off the dgrad chain)."""
    R, S = cv.weight.shape[2], cv.weight.shape[3]
    sink = sinks.target(cv.weight)
    if in_bn is None:
        with SideWork(dy, x):
            m.conv_wgrad(dy, x, R, S, stride, pad, 0, -1, sink, True)
    else:
        with SideWork(dy, x, *in_bn):
            m.conv_wgrad(dy, x, R, S, stride, pad, 0, -1, sink, True, in_bn[0], in_bn[1])


class _Bottleneck(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blk, wc, training, group, *params):
        m = _ext.require()
        proj = len(blk.shortcut) > 0
        st = blk.stride
        y1, s1 = _conv(m, x, wc.fwd(blk.conv1), 1, 0, training)
        cnt1 = (y1.numel() // y1.shape[-1]) * _world(group)
        sc1, sh1, mu1, iv1 = _BN.forward(m, s1, blk.bn1, cnt1, training, group)
        a1, f1 = _act(m, y1, sc1, sh1)
        y2, s2 = _conv(m, a1, wc.fwd(blk.conv2), st, 1, training, f1)
        cnt2 = (y2.numel() // y2.shape[-1]) * _world(group)
        sc2, sh2, mu2, iv2 = _BN.forward(m, s2, blk.bn2, cnt2, training, group)
        a2, f2 = _act(m, y2, sc2, sh2)
        y3, s3 = _conv(m, a2, wc.fwd(blk.conv3), 1, 0, training, f2)
        sc3, sh3, mu3, iv3 = _BN.forward(m, s3, blk.bn3, cnt2, training, group)
        ys = mus = ivs = None
        if proj:
            ys, ss = _conv(m, x, wc.fwd(blk.shortcut[0]), st, 0, training)
            scs, shs, mus, ivs = _BN.forward(m, ss, blk.shortcut[1], cnt2, training, group)
            om = _omask(y3, training)
            out = m.bn_apply(y3, sc3, sh3, ys, scs, shs, 1, True, mask_out=om)
        else:
            om = _omask(y3, training)
            out = m.bn_apply(y3, sc3, sh3, x, None, None, 2, True, mask_out=om)
        if training:
            fused = f1 is not None
            # the output's 1-bit ReLU mask stands in for `out` in backward
            ctx.save_for_backward(x, y1, None if fused else a1, y2, None if fused else a2, y3, ys, om, mu1, iv1,
                                  mu2, iv2, mu3, iv3, mus, ivs, sc1, sh1, sc2, sh2)
            ctx.blk, ctx.wc, ctx.group, ctx.params = blk, wc, group, params
            ctx.cnt = (cnt1, cnt2)
        return out

    @staticmethod
    def backward(ctx, dout):
        m = _ext.require()
        x, y1, a1, y2, a2, y3, ys, out, mu1, iv1, mu2, iv2, mu3, iv3, mus, ivs, sc1, sh1, sc2, sh2 = ctx.saved_tensors
        f1 = (sc1, sh1) if a1 is None else None
        f2 = (sc2, sh2) if a2 is None else None
        blk, wc, group = ctx.blk, ctx.wc, ctx.group
        cnt1, cnt2 = ctx.cnt
        st = blk.stride
        H, W = x.shape[1], x.shape[2]
        dout = dout.contiguous()
        proj = ys is not None
        if proj:
            dy3, dys, _ = _bn_bwd(m, dout, out, y3, mu3, iv3, blk.bn3, cnt2, group, ys, mus, ivs, blk.shortcut[1])
            dz = None
        else:
            # identity shortcut: dz = dout·mask is folded into the last dgrad epilogue
            dy3, _, _ = _bn_bwd(m, dout, out, y3, mu3, iv3, blk.bn3, cnt2, group)
        _wgrad(m, dy3, y2 if f2 else a2, blk.conv3, 1, 0, f2)
        da2 = m.conv_dgrad(dy3, wc.dgrad(blk.conv3), y2.shape[1], y2.shape[2], 1, 0)
        # ReLU mask recomputed from y (read anyway) instead of reading the activation
        dy2, _, _ = _bn_bwd(m, da2, None, y2, mu2, iv2, blk.bn2, cnt2, group, mask=(sc2, sh2))
        _wgrad(m, dy2, y1 if f1 else a1, blk.conv2, st, 1, f1)
        da1 = m.conv_dgrad(dy2, wc.dgrad(blk.conv2), H, W, st, 1)
        dy1, _, _ = _bn_bwd(m, da1, None, y1, mu1, iv1, blk.bn1, cnt1, group, mask=(sc1, sh1))
        _wgrad(m, dy1, x, blk.conv1, 1, 0)
        if proj:
            _wgrad(m, dys, x, blk.shortcut[0], st, 0)
            dx = m.conv_dgrad(dys, wc.dgrad(blk.shortcut[0]), H, W, st, 0)
            dx = m.conv_dgrad(dy1, wc.dgrad(blk.conv1), H, W, 1, 0, -1, dx, dx)
        else:
            dx = m.conv_dgrad(dy1, wc.dgrad(blk.conv1), H, W, 1, 0, -1, None, dout, out)
        sinks.notify(ctx.params)
        return (dx, None, None, None, None) + (None,) * len(ctx.params)


class _Basic(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blk, wc, training, group, *params):
        m = _ext.require()
        proj = len(blk.shortcut) > 0
        st = blk.stride
        y1, s1 = _conv(m, x, wc.fwd(blk.conv1), st, 1, training)
        cnt = (y1.numel() // y1.shape[-1]) * _world(group)
        sc1, sh1, mu1, iv1 = _BN.forward(m, s1, blk.bn1, cnt, training, group)
        a1, f1 = _act(m, y1, sc1, sh1)
        y2, s2 = _conv(m, a1, wc.fwd(blk.conv2), 1, 1, training, f1)
        sc2, sh2, mu2, iv2 = _BN.forward(m, s2, blk.bn2, cnt, training, group)
        ys = mus = ivs = None
        if proj:
            ys, ss = _conv(m, x, wc.fwd(blk.shortcut[0]), st, 0, training)
            scs, shs, mus, ivs = _BN.forward(m, ss, blk.shortcut[1], cnt, training, group)
            om = _omask(y2, training)
            out = m.bn_apply(y2, sc2, sh2, ys, scs, shs, 1, True, mask_out=om)
        else:
            om = _omask(y2, training)
            out = m.bn_apply(y2, sc2, sh2, x, None, None, 2, True, mask_out=om)
        if training:
            ctx.save_for_backward(x, y1, None if f1 is not None else a1, y2, ys, om, mu1, iv1, mu2, iv2, mus, ivs,
                                  sc1, sh1)
            ctx.blk, ctx.wc, ctx.group, ctx.params, ctx.cnt = blk, wc, group, params, cnt
        return out

    @staticmethod
    def backward(ctx, dout):
        m = _ext.require()
        x, y1, a1, y2, ys, out, mu1, iv1, mu2, iv2, mus, ivs, sc1, sh1 = ctx.saved_tensors
        f1 = (sc1, sh1) if a1 is None else None
        blk, wc, group, cnt = ctx.blk, ctx.wc, ctx.group, ctx.cnt
        st = blk.stride
        H, W = x.shape[1], x.shape[2]
        dout = dout.contiguous()
        proj = ys is not None
        if proj:
            dy2, dys, _ = _bn_bwd(m, dout, out, y2, mu2, iv2, blk.bn2, cnt, group, ys, mus, ivs, blk.shortcut[1])
            dz = None
        else:
            dy2, _, _ = _bn_bwd(m, dout, out, y2, mu2, iv2, blk.bn2, cnt, group)
        _wgrad(m, dy2, y1 if f1 else a1, blk.conv2, 1, 1, f1)
        da1 = m.conv_dgrad(dy2, wc.dgrad(blk.conv2), y1.shape[1], y1.shape[2], 1, 1)
        dy1, _, _ = _bn_bwd(m, da1, None, y1, mu1, iv1, blk.bn1, cnt, group, mask=(sc1, sh1))
        _wgrad(m, dy1, x, blk.conv1, st, 1)
        if proj:
            _wgrad(m, dys, x, blk.shortcut[0], st, 0)
            dx = m.conv_dgrad(dys, wc.dgrad(blk.shortcut[0]), H, W, st, 0)
            dx = m.conv_dgrad(dy1, wc.dgrad(blk.conv1), H, W, st, 1, -1, dx, dx)
        else:
            dx = m.conv_dgrad(dy1, wc.dgrad(blk.conv1), H, W, st, 1, -1, None, dout, out)
        sinks.notify(ctx.params)
        return (dx, None, None, None, None) + (None,) * len(ctx.params)


class _Stem(torch.autograd.Function):
    """conv1 + bn1 + ReLU (+ 3x3/2 max-pool for the ImageNet stem); no input gradient."""

    @staticmethod
    def forward(ctx, x, enc, wc, training, group, *params):
        m = _ext.require()
        imagenet = enc.stem == "imagenet"
        st, pad = (2, 3) if imagenet else (1, 1)
        y, s = _conv(m, x, wc.fwd(enc.conv1), st, pad, training)
        cnt = (y.numel() // y.shape[-1]) * _world(group)
        sc, sh, mu, iv = _BN.forward(m, s, enc.bn1, cnt, training, group)
        a = m.bn_apply(y, sc, sh, None, None, None, 0, True)
        # max-pool: its first-max positions (uint8) stand in for a and the pooled output in backward
        out, idx = m.maxpool_fwd_idx(a, 3, 2, 1) if imagenet else (a, None)
        if training:
            ctx.save_for_backward(x, y, idx, mu, iv, sc, sh)
            ctx.enc, ctx.group, ctx.params, ctx.cnt, ctx.geo = enc, group, params, cnt, (st, pad, imagenet)
            ctx.hw = (a.shape[1], a.shape[2])
        return out

    @staticmethod
    def backward(ctx, dout):
        m = _ext.require()
        x, y, idx, mu, iv, sc, sh = ctx.saved_tensors
        st, pad, imagenet = ctx.geo
        dout = dout.contiguous()
        da = m.maxpool_bwd_idx(idx, dout, ctx.hw[0], ctx.hw[1], 3, 2, 1) if imagenet else dout
        dy, _, _ = _bn_bwd(m, da, None, y, mu, iv, ctx.enc.bn1, ctx.cnt, ctx.group, mask=(sc, sh))
        w = ctx.enc.conv1.weight
        K, C, R, S = w.shape
        g = sinks.target(w)
        # the stem's weight gradient is the last work of the backward: on the compute stream
        # (idle from here on) it overlaps the wgrad stream's remaining queue instead of
        # waiting behind it (SDX_STEM_SIDE=1: on the side stream)
        with (SideWork(dy, x) if _STEM_SIDE else contextlib.nullcontext()):
            dwk = m.conv_wgrad(dy, x, R, S, st, pad, 0, -1)      # [K][R][S][Cp] fp32
            gk = g.permute(0, 2, 3, 1)                             # [K][R][S][C] (channels_last sink)
            if gk.is_contiguous():
                m.unpad_add(dwk, gk)
            else:
                gk.add_(dwk[..., :C])
        sinks.notify(ctx.params)
        return (None, None, None, None, None) + (None,) * len(ctx.params)


class BlockLink:
    """Hand-off between two consecutive native blocks i -> i+1 (one per forward pass).

    ``prev``: block i's ``[y_last, mean_last, y_shortcut|-, mean_shortcut|-, out bitmask]``,
    read by block i+1's backward, whose final dgrad (the kernel that stores dL/d out_i)
    emits block i's output-BN backward sums in its epilogue; ``slab`` carries them back to
    block i's backward, which then skips its separate reduction pass over dout."""
    __slots__ = ("prev", "slab")

    def __init__(self):
        self.prev = None
        self.slab = None


class BlockChain:
    """Threads :class:`BlockLink` objects through one encoder forward."""
    __slots__ = ("last",)

    def __init__(self):
        self.last = None


class _NativeBlock(torch.autograd.Function):
    """Whole residual block through the native executor (csrc/bindings/conv_bn_ops.cpp
    ``block_fwd`` / ``block_bwd``): one host call per block and direction instead of
    ~12 / ~20 Python-level kernel calls. Same kernels and math as :class:`_Bottleneck` /
    :class:`_Basic` (materialised internal activations, ReLU masks from y in backward,
    side-stream wgrads). SyncBN: ``comm_h`` is a native small-communicator handle
    (parallel/comm.py ``native_small_comm``); the executor all-reduces every BN's sums
    itself, in place on the compute stream (0 = single-process statistics)."""

    @staticmethod
    def forward(ctx, x, blk, wc, training, info, comm_h, link_in, link_out, fold_fwd, *params):
        m = _ext.require()
        convs, bns, bottle, proj = info
        bn0 = bns[0]
        bn_list = []
        for bn in bns:
            bn_list += [bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var]
        # a projection block's shortcut conv runs on the wgrad side stream (idle in forward)
        from . import streams
        side = streams.side(x.device).cuda_stream if (proj and training and SC_SIDE and streams.ENABLED and x.is_cuda) \
            else 0
        r = m.block_fwd(x, [wc.fwd(cv) for cv in convs], bn_list, blk.stride, bottle, proj, training, bn0.eps,
                        bn0.momentum, comm_h, fold_fwd, side)
        out = r[0]
        if training:
            e = _empty(x)
            # r[7]: the block output's ReLU bitmask (1 bit/element) replaces `out` in backward
            saved = [x] + [t if t is not None else e for t in r[1:7]] + [r[7]]
            ctx.save_for_backward(*saved, *r[8:])
            ctx.blk, ctx.wc, ctx.info, ctx.params, ctx.comm_h = blk, wc, info, params, comm_h
            ctx.link_in, ctx.link_out = link_in, link_out
            ctx.fold = 0   # conv weights folded in backward: 0, 1 (conv3) or 2 (conv3 + shortcut)
            if link_out is not None:
                nconv = 3 if bottle else 2
                st = r[8:]
                # r[5] is None for a forward-folded BN3 (y3 never stored): the next block's final
                # dgrad then leaves two slab rows for Σdz·y3 (block_bwd)
                link_out.prev = [(r[5] if r[5] is not None else e) if bottle else r[3], st[4 * (nconv - 1) + 2],
                                 r[6] if proj else e, st[4 * nconv + 2] if proj else _empty_f(x), r[7]]
                rows = r[0].shape[0] * r[0].shape[1] * r[0].shape[2]
                if fold_fwd or _fold_eligible(convs, bottle, proj, rows):
                    # BN3 fold: the next block's final dgrad stores dz = dout·[out > 0] (marker)
                    link_out.prev.append(_fold_marker(x))
                    ctx.fold = 2 if (proj and _fold_shortcut(convs, rows)) else 1
                    if FOLD_GRAM_FWD:
                        # the folded convs' input Grams (a2ᵀa2, Σa2) on the side stream, idle in
                        # forward; backward's main stream waits on the event for the column sums
                        # (coherent-rounding correction of the fold bias, bnfold.hip)
                        from . import streams
                        side = streams.side(x.device).cuda_stream if streams.ENABLED else 0
                        ctx.grams = m.fold_gram(r[4], side)[:2] + (m.fold_gram(x, side)[:2] if ctx.fold == 2 else [])
                        if side:
                            ctx.gram_ev = torch.cuda.Event()
                            ctx.gram_ev.record(streams.side(x.device))
        return out

    @staticmethod
    def backward(ctx, dout):
        m = _ext.require()
        convs, bns, bottle, proj = ctx.info
        t = ctx.saved_tensors
        wc = ctx.wc
        bng = []
        for bn in bns:
            bng += [bn.weight.detach(), sinks.target(bn.weight), sinks.target(bn.bias)]
        from . import streams
        side = streams.side(dout.device).cuda_stream if streams.ENABLED else 0
        lin, lout = ctx.link_in, ctx.link_out
        in_slab = lout.slab if lout is not None else None
        prev = lin.prev if (lin is not None and lin.prev is not None) else []
        nfold = getattr(ctx, "fold", 0)
        fold_w = [wc.fwd(cv) for cv in convs[2:2 + nfold]] + (getattr(ctx, "grams", None) or [])
        ev = getattr(ctx, "gram_ev", None)
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        dx, pslab = m.block_bwd(dout.contiguous(), list(t[:8]), list(t[8:]), [wc.dgrad(cv) for cv in convs],
                                [sinks.target(cv.weight) for cv in convs], bng, ctx.blk.stride, bottle, proj, side,
                                ctx.comm_h, in_slab, prev, fold_w)
        if lout is not None:
            lout.slab = lout.prev = None
        if lin is not None:
            lin.slab = pslab if (pslab is not None and pslab.numel() > 0) else None
        sinks.notify(ctx.params)
        return (dx, None, None, None, None, None, None, None, None) + (None,) * len(ctx.params)


_EMPTY = {}
_MARK = {}

# BN3 fold of identity bottlenecks (csrc/kernels/bnfold.hip): dy3 = A·dz + D·y3 + E is never
# materialised — conv3's dgrad runs on dz with diag(A)·W3 plus the fold term
# T = a2·(W3ᵀ·diag(D)·W3) + Eᵀ·W3 added in its epilogue, and dW3 is rebuilt from dzᵀ·a2 and a2ᵀ·a2.
# Applied where conv3's input width K is at most SDX_BN3_FOLD_MAXK (the fold matrices cost C·K²;
# the elementwise pass it removes costs rows·C): layers 1-2 of the CIFAR ResNet-50.
# The fold's addend T enters conv3's dgrad accumulators before the bf16 rounding
# (GemmEpi::add_pre): added after it, T was swamped and the layer-1 BN2 gradients drifted
# at 512 views (l1.1 bn2.bias 0.32 vs 0.17 rel to fp32); with it they are at 0.166 vs 0.170
# materialised (tools/fold_bn_probe.py, profiles/bn3_fold_r2.txt).
BN3_FOLD = os.environ.get("SDX_BN3_FOLD", "1") != "0"
BN3_FOLD_MAXK = int(os.environ.get("SDX_BN3_FOLD_MAXK", "512"))
# the fold's fixed cost grows as K² (its C x K x K matrices, the K x K Gram), the pass it
# removes as rows: fold when rows >= MIN_ROWS_PER_K2 · K². CIFAR 512 views: layers 1-2
# (128, 8 rows per K²) fold, layer 3 (0.5) does not; 224x224 1024 views: layers 1-3
BN3_FOLD_ROWS_PER_K2 = float(os.environ.get("SDX_BN3_FOLD_ROWS_PER_K2", "2"))
# the fold's Gram a2ᵀ·a2 and column sums computed at forward time on the side stream; the
# column sums also feed the mean(a2) part of the fold bias's rounding correction. Opt-in:
# with the accumulator pre-add the correction is not needed (full-batch worst 0.033 rel either
# way) and Grams in backward are faster (12.53 vs 12.60 ms, profiles/bn3_fold_r2.txt)
FOLD_GRAM_FWD = os.environ.get("SDX_FOLD_GRAM_FWD", "0") != "0"
# forward half of the fold (block_fwd fold_fwd, default on): conv3 twice — BN3 statistics, then
# BN3 + residual + ReLU in its epilogue — so y3 is never stored; Σdz·y3 in backward from
# W3 and dzᵀ·a2. Needs the next block's dgrad statistics hand-off (SDX_DGRAD_BNSTAT)
FOLD_FWD = os.environ.get("SDX_BN3_FOLD_FWD", "1") != "0"
DGRAD_BNSTAT = os.environ.get("SDX_DGRAD_BNSTAT", "1") != "0"


def _fold_eligible(convs, bottle, proj, rows) -> bool:
    """BN3 of a bottleneck (identity or projection); see _fold_shortcut for the shortcut BN."""
    if not (BN3_FOLD and bottle):
        return False
    k = convs[2].in_channels
    if not (convs[2].kernel_size == (1, 1) and k <= BN3_FOLD_MAXK
            and rows >= BN3_FOLD_ROWS_PER_K2 * k * k):
        return False
    return True


def _fold_shortcut(convs, rows) -> bool:
    """A projection bottleneck's 1x1 shortcut BN folds the same way over the block input when
    the shortcut has stride 1 (else its dys is materialised from the already-masked dz)."""
    sc = convs[3]
    ks = sc.in_channels
    return (sc.kernel_size == (1, 1) and sc.stride == (1, 1) and ks <= BN3_FOLD_MAXK
            and rows >= BN3_FOLD_ROWS_PER_K2 * ks * ks)


def _fold_marker(like):
    t = _MARK.get(like.device)
    if t is None:
        t = _MARK[like.device] = torch.ones(1, dtype=torch.uint8, device=like.device)
    return t


def _empty_f(like):
    return _empty(torch.empty(0, dtype=torch.float32, device=like.device))


def _empty(like):
    e = _EMPTY.get(like.device)
    if e is None:
        e = _EMPTY[like.device] = torch.empty(0, dtype=like.dtype, device=like.device)
    return e


NATIVE_EXEC = os.environ.get("SDX_NATIVE_EXEC", "1") != "0"
# projection blocks: the shortcut conv runs on the (forward-idle) side stream, concurrently
# with conv1 -> bn1 -> conv2 -> ...; its BN finalize stays on the compute stream
SC_SIDE = os.environ.get("SDX_SC_SIDE", "1") != "0"


def _block_info(blk):
    """(convs, bns, bottleneck?, projection?) and the parameter list, cached on the module."""
    info = getattr(blk, "_sdx_info", None)
    if info is None:
        bottle = hasattr(blk, "conv3")
        proj = len(blk.shortcut) > 0
        convs = [blk.conv1, blk.conv2] + ([blk.conv3] if bottle else []) + ([blk.shortcut[0]] if proj else [])
        bns = [blk.bn1, blk.bn2] + ([blk.bn3] if bottle else []) + ([blk.shortcut[1]] if proj else [])
        info = ((convs, bns, bottle, proj), [p for p in blk.parameters()])
        blk._sdx_info = info
    return info


def _native_comm(group, blk_info) -> int:
    """-1: Python block path; else the executor's SyncBN handle (0 = no SyncBN)."""
    bns = blk_info[1]
    if not (NATIVE_EXEC and not FUSE_PROLOGUE and bns[0].momentum is not None
            and all(bn.affine and bn.track_running_stats for bn in bns)):
        return -1
    if group is None:
        return 0
    h = comm.native_small_comm(group)
    return h if h else -1


def block_params(mod) -> List[torch.nn.Parameter]:
    info = getattr(mod, "_sdx_info", None)
    return list(info[1]) if info is not None else [p for p in mod.parameters()]


def _fold_fwd(x, info, training, next_native) -> bool:
    """Forward half of the BN3 fold (block_fwd fold_fwd): bottlenecks that fold their BN3
    backward AND whose successor is a native block (its final dgrad supplies the slab the
    folded backward needs, since y3 is not kept). Identity blocks add x in conv3's epilogue;
    projection blocks (any stride) add BN_s(ys), the shortcut BN applied in the same epilogue."""
    convs, bns, bottle, proj = info
    if not (FOLD_FWD and training and next_native and bottle and DGRAD_BNSTAT):
        return False
    if not proj and convs[1].stride != (1, 1):
        return False
    s = convs[1].stride[0]
    rows = (x.shape[0] * ((x.shape[1] - 1) // s + 1) * ((x.shape[2] - 1) // s + 1))
    return _fold_eligible(convs, bottle, proj, rows)


def bottleneck(x, blk, wc, training: bool, group=None, chain: Optional[BlockChain] = None,
               next_native: bool = False):
    """``next_native``: the block that consumes this one's output is a native block too
    (set by the executor for every block but the encoder's last)."""
    info, params = _block_info(blk)
    h = _native_comm(group, info)
    if h >= 0:
        lin = chain.last if chain is not None else None
        lout = BlockLink() if (chain is not None and training) else None
        if chain is not None:
            chain.last = lout
        ff = lout is not None and _fold_fwd(x, info, training, next_native)
        return _NativeBlock.apply(x, blk, wc, training, info, h, lin, lout, ff, *params)
    if chain is not None:
        chain.last = None
    return _Bottleneck.apply(x, blk, wc, training, group, *params)


def basic(x, blk, wc, training: bool, group=None, chain: Optional[BlockChain] = None):
    info, params = _block_info(blk)
    h = _native_comm(group, info)
    if h >= 0:
        lin = chain.last if chain is not None else None
        lout = BlockLink() if (chain is not None and training) else None
        if chain is not None:
            chain.last = lout
        return _NativeBlock.apply(x, blk, wc, training, info, h, lin, lout, False, *params)
    if chain is not None:
        chain.last = None
    return _Basic.apply(x, blk, wc, training, group, *params)


def stem(x, enc, wc, training: bool, group=None):
    ps = [enc.conv1.weight, enc.bn1.weight, enc.bn1.bias]
    return _Stem.apply(x, enc, wc, training, group, *ps)
