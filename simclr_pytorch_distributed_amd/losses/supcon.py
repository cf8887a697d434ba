"""SupCon / SimCLR (NT-Xent) contrastive loss.

Reference semantics (losses.py:17-93): for each anchor ``i`` and contrast ``j != i``
``s_ij = a_i·c_j / τ``; ``ℓ_i = -(τ/τ_base)·mean_{p∈P(i)} (s_ip - log Σ_{j≠i} exp s_ij)``;
the loss is the mean of ``ℓ_i`` over anchors. ``P(i)`` = other views of the same sample
(SimCLR) or same-label contrasts (SupCon).

This module re-expresses the loss in a *row-block* form: anchors are identified by the
index of their own row in the contrast matrix (``self_idx``) and positives by an integer
``key`` per row (sample id for SimCLR, label for SupCon), so the N×N mask is never
materialised. That row form is what the fused gfx950 kernel (``ops/contrastive.py``)
implements, and what lets each rank own only its anchors while contrasting against
the globally gathered matrix.

Deviation: anchors with no positive (possible only for SupCon with a unique label in
``contrast_mode='one'``) contribute 0 instead of the reference's NaN.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..parallel import comm


def supcon_rows_reference(A: torch.Tensor, C: torch.Tensor, self_idx: torch.Tensor,
                          akey: torch.Tensor, ckey: torch.Tensor, temperature: float,
                          base_temperature: float) -> torch.Tensor:
    """Per-anchor loss ℓ_i (pure torch, fp32; CPU path and kernel oracle)."""
    dt = torch.promote_types(torch.promote_types(A.dtype, C.dtype), torch.float32)
    A = A.to(dt)
    C = C.to(dt)
    logits = A @ C.t() / temperature
    n = C.shape[0]
    cols = torch.arange(n, device=C.device)
    not_self = cols[None, :] != self_idx[:, None].long()
    pos = (akey[:, None] == ckey[None, :]) & not_self
    logits = logits.masked_fill(~not_self, float("-inf"))
    lse = torch.logsumexp(logits, dim=1)
    logits0 = logits.masked_fill(~not_self, 0.0)
    cnt = pos.sum(1)
    psum = (logits0 * pos).sum(1)
    mean_pos = torch.where(cnt > 0, psum / cnt.clamp_min(1), lse)
    return -(temperature / base_temperature) * (mean_pos - lse)


def _native_available(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    from ..ops import contrastive
    return contrastive.supported(t)


def row_normalize(x: torch.Tensor, backend: str = "auto") -> torch.Tensor:
    """F.normalize(x, dim=1) — one fused launch each way on GPU (ops/contrastive.py)."""
    if backend != "torch" and x.is_cuda:
        from ..ops import contrastive
        return contrastive.row_normalize(x)
    return F.normalize(x, dim=1)


def supcon_rows_loss(A, C, self_idx, akey, ckey, temperature, base_temperature, scale: float,
                     backend: str = "auto") -> torch.Tensor:
    """``scale * Σ_i ℓ_i`` over the given anchor rows (differentiable w.r.t. A and C)."""
    use_native = backend == "native" or (backend == "auto" and _native_available(C))
    if use_native:
        from ..ops import contrastive
        return contrastive.supcon_rows_loss(A, C, self_idx, akey, ckey, temperature,
                                            base_temperature, scale)
    return scale * supcon_rows_reference(A, C, self_idx, akey, ckey, temperature, base_temperature).sum()


class SupConLoss(nn.Module):
    """Drop-in for the reference ``SupConLoss`` (losses.py:7-93), same arguments."""

    def __init__(self, temperature: float = 0.07, contrast_mode: str = "all",
                 base_temperature: float = 0.07, backend: str = "auto"):
        super().__init__()
        self.temperature = temperature
        self.contrast_mode = contrast_mode
        self.base_temperature = base_temperature
        self.backend = backend

    def forward(self, features: torch.Tensor, labels: Optional[torch.Tensor] = None,
                mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if features.dim() < 3:
            raise ValueError("`features` needs to be [bsz, n_views, ...],"
                             "at least 3 dimensions are required")
        if features.dim() > 3:
            features = features.view(features.shape[0], features.shape[1], -1)
        bsz, n_views = features.shape[0], features.shape[1]
        if labels is not None and mask is not None:
            raise ValueError("Cannot define both `labels` and `mask`")
        if mask is not None:
            return self._dense_mask_forward(features, mask.float())
        if labels is not None:
            labels = labels.contiguous().view(-1)
            if labels.shape[0] != bsz:
                raise ValueError("Num of labels does not match num of features")
            key = labels.to(torch.int32)
        else:
            key = torch.arange(bsz, device=features.device, dtype=torch.int32)
        if self.contrast_mode not in ("one", "all"):
            raise ValueError(f"Unknown mode: {self.contrast_mode}")
        contrast = torch.cat(torch.unbind(features, dim=1), dim=0)  # [n_views*bsz, d]
        ckey = key.repeat(n_views)
        if self.contrast_mode == "one":
            anchor, akey = features[:, 0], key
            self_idx = torch.arange(bsz, device=features.device, dtype=torch.int32)
        else:
            anchor, akey = contrast, ckey
            self_idx = torch.arange(n_views * bsz, device=features.device, dtype=torch.int32)
        n_anchor = anchor.shape[0]
        return supcon_rows_loss(anchor, contrast, self_idx, akey, ckey, self.temperature,
                                self.base_temperature, 1.0 / n_anchor, self.backend)

    def _dense_mask_forward(self, features, mask):
        """Arbitrary [bsz, bsz] mask: the reference's dense formulation (losses.py:50-93)."""
        device = features.device
        bsz, n_views = features.shape[:2]
        contrast = torch.cat(torch.unbind(features, dim=1), dim=0)
        if self.contrast_mode == "one":
            anchor, anchor_count = features[:, 0], 1
        elif self.contrast_mode == "all":
            anchor, anchor_count = contrast, n_views
        else:
            raise ValueError(f"Unknown mode: {self.contrast_mode}")
        logits = anchor @ contrast.t() / self.temperature
        logits = logits - logits.max(dim=1, keepdim=True)[0].detach()
        mask = mask.to(device).repeat(anchor_count, n_views)
        logits_mask = torch.ones_like(mask)
        idx = torch.arange(bsz * anchor_count, device=device)
        logits_mask[idx, idx] = 0
        mask = mask * logits_mask
        exp_logits = torch.exp(logits) * logits_mask
        log_prob = logits - torch.log(exp_logits.sum(1, keepdim=True))
        mean_log_prob_pos = (mask * log_prob).sum(1) / mask.sum(1)
        loss = -(self.temperature / self.base_temperature) * mean_log_prob_pos
        return loss.view(anchor_count, bsz).mean()


class DistributedContrastiveLoss(nn.Module):
    """Global-negatives contrastive loss with row ownership (replaces main_supcon.py:268-293).

    Input: this rank's *raw* projections ``feats`` ``[n_views*B_l, d]`` in view-major
    order (``cat([view1, view2])`` as the reference builds ``images``) and optional
    ``labels`` ``[B_l]``. The rank L2-normalises its rows, all-gathers the normalised
    matrix (backward: reduce-scatter), and evaluates ℓ_i for its own anchors only
    against all ``n_views*B`` contrasts. Returns ``Σ_{i local} ℓ_i / N_anchor_global``, so
    the sum over ranks is the reference's global loss and each rank's gradient is the
    exact gradient of that global loss w.r.t. its own rows (the reference's DDP-averaged
    gradient is then reproduced by mean-reducing parameter gradients).
    """

    def __init__(self, method: str = "SimCLR", temperature: float = 0.5, base_temperature: float = 0.07,
                 contrast_mode: str = "all", n_views: int = 2, backend: str = "auto"):
        super().__init__()
        if method not in ("SimCLR", "SupCon"):
            raise ValueError(f"contrastive method not supported: {method}")
        self.method = method
        self.temperature = temperature
        self.base_temperature = base_temperature
        self.contrast_mode = contrast_mode
        self.n_views = n_views
        self.backend = backend
        self._idx_cache = {}

    def _indices(self, b_local: int, w: int, r: int, device, labels_all):
        key = (b_local, w, r, str(device), labels_all is None)
        nv = self.n_views
        if key not in self._idx_cache or labels_all is not None:
            # gathered layout: rank-major, then view, then local sample
            g = torch.arange(w * nv * b_local, device=device)
            rr = g // (nv * b_local)
            j = g % b_local
            sample = (rr * b_local + j).to(torch.int32)
            if labels_all is not None:
                lab = labels_all.view(w, b_local).to(torch.int32)
                ckey = lab[rr, j]
            else:
                ckey = sample
            base = r * nv * b_local
            if self.contrast_mode == "all":
                self_idx = torch.arange(base, base + nv * b_local, device=device, dtype=torch.int32)
            else:
                self_idx = torch.arange(base, base + b_local, device=device, dtype=torch.int32)
            akey = ckey[self_idx.long()]
            val = (self_idx, akey, ckey)
            if labels_all is None:
                self._idx_cache[key] = val
            return val
        return self._idx_cache[key]

    def forward(self, feats: torch.Tensor, labels: Optional[torch.Tensor] = None):
        w, r = comm.world_size(), comm.rank()
        nv = self.n_views
        b_local = feats.shape[0] // nv
        x = feats.to(torch.promote_types(feats.dtype, torch.float32))
        h = comm.native_gather_comm() if (w > 1 and self.backend != "torch" and x.is_cuda) else 0
        if h and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] <= 256:
            # normalised rows land in this rank's block of C, gathered in place on the
            # native RCCL communicator (backward: reduce-scatter) — no c10d call
            from ..ops.contrastive import row_normalize_gather
            C = row_normalize_gather(x, h)
            n = C[r * x.shape[0]:(r + 1) * x.shape[0]]
        else:
            h = 0
            n = row_normalize(x, self.backend)
            C = comm.all_gather_with_grad(n)
        labels_all = None
        if self.method == "SupCon":
            if labels is None:
                raise ValueError("SupCon needs labels")
            lab = labels.to(torch.int64).contiguous()
            if h:
                from ..ops import _ext
                labels_all = _ext.require().small_all_gather(h, lab)
            else:
                labels_all = comm.all_gather_tensor(lab)
        self_idx, akey, ckey = self._indices(b_local, w, r, feats.device, labels_all)
        A = n if self.contrast_mode == "all" else n[:b_local]
        n_anchor_global = A.shape[0] * w
        return supcon_rows_loss(A, C, self_idx, akey, ckey, self.temperature, self.base_temperature,
                                1.0 / n_anchor_global, self.backend)
