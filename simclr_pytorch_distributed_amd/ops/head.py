"""Projection head (reference networks/resnet_big.py:159-181: MLP Linear-ReLU-Linear or a
single Linear) as ONE autograd node on the native path.

The GEMMs are plain library GEMMs (hipBLASLt through ``torch.mm``/``addmm``) on the bf16
weights the per-step weight cache already produced (ops/weights.py: the head's Linear
layers are cached as 1x1 convs, so no per-step weight casts); weight gradients are
accumulated straight into the parameter sinks. Autograd would otherwise build ~20 nodes for this tiny region (casts, addmm, relu,
AccumulateGrad), and their host cost leaves the GPU idle between forward and backward.
Numerics: identical to ``models.executor.head_forward`` (bf16 operands and bias, fp32
accumulation, ReLU on the bf16 hidden activations).
"""
from __future__ import annotations

import torch

from . import sinks

_BF = torch.bfloat16


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    # bf16 output, accumulated into the fp32 sink by the caller (as autograd's bf16 weight
    # grad + AccumulateGrad did): ``mm(out_dtype=fp32)`` measured ~160 us of host time per
    # call on this stack, which left the GPU idle in the head region
    return torch.mm(a, b)


class _MLPHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, w1b, w2b, l1, l2, *params):
        fb = feat.to(_BF)
        h = torch.addmm(l1.bias.detach().to(_BF), fb, w1b.t())
        h.relu_()
        z = torch.addmm(l2.bias.detach().to(_BF), h, w2b.t()).float()
        ctx.save_for_backward(fb, h, w1b, w2b)
        ctx.mods = (l1, l2)
        ctx.params = params
        ctx.feat_dtype = feat.dtype
        return z

    @staticmethod
    def backward(ctx, dz):
        fb, h, w1b, w2b = ctx.saved_tensors
        l1, l2 = ctx.mods
        dzb = dz.to(_BF)
        sinks.target(l2.weight).add_(_mm_f32(dzb.t(), h))
        sinks.target(l2.bias).add_(dz.sum(0))
        dh = torch.ops.aten.threshold_backward(torch.mm(dzb, w2b), h, 0)
        sinks.target(l1.weight).add_(_mm_f32(dh.t(), fb))
        sinks.target(l1.bias).add_(dh.sum(0, dtype=torch.float32))
        dfeat = torch.mm(dh, w1b).to(ctx.feat_dtype)
        sinks.notify(ctx.params)
        return (dfeat, None, None, None, None) + (None,) * len(ctx.params)


class _LinearHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, wb, lin, *params):
        fb = feat.to(_BF)
        z = torch.addmm(lin.bias.detach().to(_BF), fb, wb.t()).float()
        ctx.save_for_backward(fb, wb)
        ctx.lin = lin
        ctx.params = params
        ctx.feat_dtype = feat.dtype
        return z

    @staticmethod
    def backward(ctx, dz):
        fb, wb = ctx.saved_tensors
        lin = ctx.lin
        dzb = dz.to(_BF)
        sinks.target(lin.weight).add_(_mm_f32(dzb.t(), fb))
        sinks.target(lin.bias).add_(dz.sum(0))
        dfeat = torch.mm(dzb, wb).to(ctx.feat_dtype)
        sinks.notify(ctx.params)
        return (dfeat, None, None) + (None,) * len(ctx.params)


def _w(wc, lin) -> torch.Tensor:
    return wc.fwd(lin).view(lin.out_features, lin.in_features)


def projection_head(feat: torch.Tensor, head, wc) -> torch.Tensor:
    """``head(feat)`` in bf16 with fp32 output, as one autograd node."""
    if isinstance(head, torch.nn.Linear):
        return _LinearHead.apply(feat, _w(wc, head), head, head.weight, head.bias)
    l1, l2 = head[0], head[2]
    return _MLPHead.apply(feat, _w(wc, l1), _w(wc, l2), l1, l2, l1.weight, l1.bias, l2.weight, l2.bias)
