"""Autograd binding of the fused contrastive-loss kernels (csrc/kernels/supcon.hip).

``supcon_rows_loss(A, C, self_idx, akey, ckey, τ, τ_base, scale)`` returns
``scale * Σ_i ℓ_i`` for the anchor rows ``A`` (rows of ``C``, the L2-normalised
contrast matrix). Forward: one split tile kernel + one finalize kernel; backward: two
tile kernels (dA, dC). The upstream gradient stays on device (no host sync), so the op
is hipGraph-capturable. Oracle: ``losses.supcon.supcon_rows_reference``.
"""
from __future__ import annotations

import torch

from . import _ext

_SUPPORTED_D = (64, 128, 256)


def supported(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dim() == 2 and t.shape[1] in _SUPPORTED_D and _ext.available()


class _SupConRows(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, C, self_idx, akey, ckey, temperature, base_temperature, scale):
        m = _ext.require()
        A32 = A.float().contiguous()
        C32 = C.float().contiguous()
        si = self_idx.to(torch.int32).contiguous()
        ak = akey.to(torch.int32).contiguous()
        ck = ckey.to(torch.int32).contiguous()
        ratio = temperature / base_temperature
        loss, lse, invcnt, row_loss = m.supcon_fwd(A32, C32, si, ak, ck, 1.0 / temperature, ratio, scale)
        ctx.save_for_backward(A32, C32, si, ak, ck, lse, invcnt)
        ctx.w = scale * ratio / temperature
        ctx.inv_temp = 1.0 / temperature
        ctx.dtypes = (A.dtype, C.dtype)
        # one rank, contrast_mode "all": the anchors ARE the contrasts (one tensor) -> the
        # backward sums dA + dC inside its split reduction
        ctx.same = A is C and A32.shape[0] == C32.shape[0]
        ctx.mark_non_differentiable(row_loss)
        # no zero-filled gradient for the per-row output (one fill kernel less per step)
        ctx.set_materialize_grads(False)
        return loss.view(()), row_loss

    @staticmethod
    def backward(ctx, g, _g_rows):
        if g is None:
            return (None,) * 8
        m = _ext.require()
        A32, C32, si, ak, ck, lse, invcnt = ctx.saved_tensors
        gl = g.float().reshape(1).contiguous()
        if ctx.same:
            dX = m.supcon_bwd_sum(A32, si, ak, ck, lse, invcnt, gl, ctx.inv_temp, ctx.w)
            return dX.to(ctx.dtypes[0]), None, None, None, None, None, None, None
        dA, dC = m.supcon_bwd(A32, C32, si, ak, ck, lse, invcnt, gl, ctx.inv_temp, ctx.w)
        return dA.to(ctx.dtypes[0]), dC.to(ctx.dtypes[1]), None, None, None, None, None, None


class _RowNorm(torch.autograd.Function):
    """F.normalize(x, dim=1, eps) on fp32 rows as one launch each way (csrc/kernels/featnorm.hip)."""

    @staticmethod
    def forward(ctx, x, eps):
        y, norms = _ext.require().rownorm_fwd(x.contiguous(), eps)
        ctx.save_for_backward(y, norms)
        ctx.eps = eps
        return y

    @staticmethod
    def backward(ctx, dy):
        y, norms = ctx.saved_tensors
        return _ext.require().rownorm_bwd(dy.contiguous(), y, norms, ctx.eps), None


class _RowNormGather(torch.autograd.Function):
    """Row L2 normalisation written straight into this rank's block of the gathered
    contrast matrix, all-gathered in place on a native communicator (RCCL; an emulated
    one in single-GPU tests); backward: reduce-scatter of dC to the row owners, then the
    normalisation gradient (csrc/bindings/comm_ops.cpp rownorm_gather[_bwd])."""

    @staticmethod
    def forward(ctx, x, handle, eps):
        C, norms = _ext.require().rownorm_gather(handle, x.contiguous(), eps)
        ctx.save_for_backward(C, norms)
        ctx.meta = (handle, eps, x.shape[0])
        return C

    @staticmethod
    def backward(ctx, gC):
        C, norms = ctx.saved_tensors
        handle, eps, n = ctx.meta
        m = _ext.require()
        r = m.small_comm_rank(handle)
        return m.rownorm_gather_bwd(handle, gC.contiguous(), C[r * n:(r + 1) * n], norms, eps), None, None


def row_normalize_gather(x: torch.Tensor, handle: int, eps: float = 1e-12) -> torch.Tensor:
    """``all_gather(F.normalize(x, dim=1))`` (rank-major) with reduce-scatter backward."""
    return _RowNormGather.apply(x, handle, eps)


def row_normalize(x: torch.Tensor, eps: float = 1e-12) -> torch.Tensor:
    """Row L2 normalisation (reference main_supcon.py:283, ``F.normalize(dim=1)``)."""
    if x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and x.shape[1] <= 256 and _ext.available():
        return _RowNorm.apply(x, eps)
    return torch.nn.functional.normalize(x, dim=1, eps=eps)


def supcon_rows_loss(A, C, self_idx, akey, ckey, temperature, base_temperature, scale, return_rows=False):
    loss, rows = _SupConRows.apply(A, C, self_idx, akey, ckey, float(temperature), float(base_temperature),
                                   float(scale))
    return (loss, rows) if return_rows else loss
