"""Autograd binding of the implicit-GEMM MFMA convolution (csrc/kernels/igemm.hip).

Activations are NHWC bf16; master weights stay fp32 in the module's parameter (shape
``[Cout, Cin, R, S]``, same as the reference's ``nn.Conv2d``; stored channels_last so
the physical layout is KRSC and the fp32 weight-gradient kernel writes it directly).

``conv2d_nhwc(x, weight, stride, pad, stats=True)`` returns ``(y, sums)`` where ``sums``
is the fp64 ``[2, Cout]`` (Σy, Σy²) of the stored output, produced by the convolution
epilogue for the BatchNorm that follows (training) — or ``None``.
"""
from __future__ import annotations

import torch

from . import _ext


def weight_krsc_bf16(weight: torch.Tensor, cin_pad: int = 0) -> torch.Tensor:
    """fp32 [K,C,R,S] (any memory format) -> bf16 contiguous [K,R,S,C(+pad)]."""
    w = weight.detach().permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
    if cin_pad:
        w = torch.nn.functional.pad(w, (0, cin_pad)).contiguous()
    return w


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, pad, want_stats, cin_pad):
        m = _ext.require()
        wk = weight_krsc_bf16(weight, cin_pad)
        y, slab = m.conv_fwd(x, wk, stride, pad, want_stats, -1)
        sums = m.bn_stats_reduce(slab) if want_stats else None
        ctx.save_for_backward(x, wk)
        ctx.geom = (x.shape[1], x.shape[2], weight.shape[2], weight.shape[3], stride, pad, cin_pad)
        ctx.w_dtype = weight.dtype
        if sums is not None:
            ctx.mark_non_differentiable(sums)
        return y, sums

    @staticmethod
    def backward(ctx, dy, _dsums):
        m = _ext.require()
        x, wk = ctx.saved_tensors
        H, W, R, S, stride, pad, cin_pad = ctx.geom
        dy = dy.contiguous()
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wt = wk.permute(3, 1, 2, 0).contiguous()        # [C][R][S][K]
            dx = m.conv_dgrad(dy, wt, H, W, stride, pad, -1)
        if ctx.needs_input_grad[1]:
            dwk = m.conv_wgrad(dy, x, R, S, stride, pad, 0, -1)   # fp32 [K][R][S][C]
            if cin_pad:
                dwk = dwk[..., : dwk.shape[-1] - cin_pad]
            dw = dwk.permute(0, 3, 1, 2)                          # [K][C][R][S] view, channels_last strides
        return dx, dw, None, None, None, None


def conv2d_nhwc(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, pad: int = 0, stats: bool = True,
                cin_pad: int = 0):
    return _Conv.apply(x, weight, stride, pad, stats, cin_pad)
