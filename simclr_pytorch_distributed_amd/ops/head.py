"""Projection head (reference networks/resnet_big.py:159-181: MLP Linear-ReLU-Linear or a
single Linear) as ONE autograd node on the native path.

Both directions are one host call into the C++ head executor (csrc/bindings/head_ops.cpp),
which runs the GEMMs as 1x1 implicit GEMMs of the hand-written MFMA kernel (igemm.hip)
with fused epilogues: bias + ReLU on the fp32 accumulators, fp32 feature output, ReLU
backward fused into the hidden-gradient store together with its column sums (the hidden
bias gradient). Weight and bias gradients are accumulated straight into the parameter
sinks. The bf16 weights come from the per-step weight cache (ops/weights.py caches the
head's Linear layers as 1x1 convs, in both the forward and the transposed layout).
Numerics: bf16 operands, fp32 accumulation, fp32 biases, bf16 hidden activation, fp32
output — the reference computed under autocast, with the bias added before rounding.
"""
from __future__ import annotations

import os

import torch

from . import _ext, sinks


_HEAD_SIDE = os.environ.get("SDX_HEAD_SIDE", "1") != "0"


def _side(t: torch.Tensor) -> int:
    """the wgrad side stream's handle for the head's weight gradients (0: none). The current
    backward pass then ends with a join (compute stream behind the side stream), so the
    parameter gradients are complete for whatever runs after ``backward()`` on the compute
    stream, not only for the optimizer step (which joins as well)."""
    from . import streams
    if not (_HEAD_SIDE and streams.ENABLED and t.is_cuda):
        return 0
    dev = t.device
    main, side = torch.cuda.current_stream(dev), streams.side(dev)   # (this node's stream)

    def _join():
        main.wait_stream(side)
        streams.release()

    torch.autograd.Variable._execution_engine.queue_callback(_join)
    return side.cuda_stream


class _MLPHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, w1b, w2b, w1t, w2t, l1, l2, *params):
        z, fb, h = _ext.require().head_fwd(feat, w1b, l1.bias.detach(), w2b, l2.bias.detach())
        ctx.save_for_backward(fb, h, w1t, w2t)
        ctx.mods = (l1, l2)
        ctx.params = params
        ctx.feat_dtype = feat.dtype
        return z

    @staticmethod
    def backward(ctx, dz):
        fb, h, w1t, w2t = ctx.saved_tensors
        l1, l2 = ctx.mods
        t = sinks.target
        dfeat = _ext.require().head_bwd(dz.float(), fb, h, w1t, w2t, t(l1.weight), t(l1.bias), t(l2.weight),
                                        t(l2.bias), _side(dz))
        sinks.notify(ctx.params)
        return (dfeat.to(ctx.feat_dtype), None, None, None, None, None, None) + (None,) * len(ctx.params)


class _LinearHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, wb, wt, lin, *params):
        z, fb, _ = _ext.require().head_fwd(feat, wb, lin.bias.detach())
        ctx.save_for_backward(fb, wt)
        ctx.lin = lin
        ctx.params = params
        ctx.feat_dtype = feat.dtype
        return z

    @staticmethod
    def backward(ctx, dz):
        fb, wt = ctx.saved_tensors
        lin = ctx.lin
        dfeat = _ext.require().head_bwd(dz.float(), fb, None, wt, None, sinks.target(lin.weight),
                                        sinks.target(lin.bias))
        sinks.notify(ctx.params)
        return (dfeat.to(ctx.feat_dtype), None, None, None) + (None,) * len(ctx.params)


def _w(wc, lin) -> torch.Tensor:
    return wc.fwd(lin).view(lin.out_features, lin.in_features)


def _wt(wc, lin) -> torch.Tensor:
    return wc.dgrad(lin).view(lin.in_features, lin.out_features)


def projection_head(feat: torch.Tensor, head, wc) -> torch.Tensor:
    """``head(feat)`` in bf16 with fp32 output, as one autograd node."""
    if isinstance(head, torch.nn.Linear):
        return _LinearHead.apply(feat, _w(wc, head), _wt(wc, head), head, head.weight, head.bias)
    l1, l2 = head[0], head[2]
    return _MLPHead.apply(feat, _w(wc, l1), _w(wc, l2), _wt(wc, l1), _wt(wc, l2), l1, l2, l1.weight, l1.bias,
                          l2.weight, l2.bias)
