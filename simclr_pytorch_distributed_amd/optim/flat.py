"""Flat parameter / gradient storage and fused optimizers.

All trainable parameters of a model are re-homed into ONE contiguous fp32 buffer and
their ``.grad`` into a second one (views keep each parameter's shape and memory format,
e.g. channels_last conv weights). Consequences, MI355X-first:

* the optimizer step is one streaming kernel (``sgd_step`` / ``lars_step`` in
  csrc/kernels/optim.hip) instead of 163 tensor launches (reference: util.py:79-84);
* data-parallel gradient buckets are contiguous slices of the flat gradient buffer, so
  RCCL all-reduces them in place (no flatten/unflatten copies; parallel/ddp.py);
* ``zero_grad`` is one memset.

Segments are laid out in *reverse* registration order (≈ the order backward produces
gradients) and padded to 4096 elements (LARS per-tensor chunks never straddle).

The optimizers keep the ``torch.optim`` surface the engine needs (``param_groups[0]['lr']``,
``state_dict``/``load_state_dict`` in torch.optim.SGD format for checkpoint
compatibility with the reference, util.py:87-96).
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ..ops import _ext

SEG_ALIGN = 4096


class FlatParams:
    def __init__(self, model: torch.nn.Module, device=None, align: int = SEG_ALIGN):
        self.model = model
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        device = device or self.params[0].device
        order = list(reversed(range(len(self.params))))   # backward order
        offsets = [0] * len(self.params)
        off = 0
        for i in order:
            offsets[i] = off
            n = self.params[i].numel()
            off += (n + align - 1) // align * align
        self.total = off
        self.offsets = offsets
        self.order = order
        self.flat = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        for i, p in enumerate(self.params):
            view = self._view(self.flat, i)
            view.copy_(p.detach())
            p.data = view
            p.grad = self._view(self.grad, i)

    def _view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        p = self.params[i]
        n = p.numel()
        seg = buf[self.offsets[i]:self.offsets[i] + n]
        if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
            K, C, R, S = p.shape
            return seg.view(K, R, S, C).permute(0, 3, 1, 2)
        return seg.view(p.shape)

    def reattach_grads(self):
        """Re-point ``.grad`` at the flat buffer (after someone set it to None)."""
        for i, p in enumerate(self.params):
            if p.grad is None or p.grad.data_ptr() != self._view(self.grad, i).data_ptr():
                g = self._view(self.grad, i)
                if p.grad is not None:
                    g.copy_(p.grad)
                p.grad = g

    def zero_grad(self):
        # one runtime fill on the step stream (hipMemsetAsync), not a torch FillFunctor kernel
        if self.grad.is_cuda and _ext.available():
            _ext.require().zero_async(self.grad)
        else:
            self.grad.zero_()

    def segment_table(self):
        offs = [self.offsets[i] for i in self.order]
        adapt = [1 if self.params[i].dim() > 1 else 0 for i in self.order]
        return offs, adapt


class _FlatOptimizer:
    def __init__(self, flat: FlatParams, lr: float, momentum: float, weight_decay: float):
        self.flat = flat
        self.momentum = momentum
        self.weight_decay = weight_decay
        self.param_groups = [dict(lr=lr, momentum=momentum, weight_decay=weight_decay, dampening=0,
                                  nesterov=False, params=flat.params)]
        self.buf = torch.zeros_like(flat.flat)
        self.lr_t = torch.full((1,), lr, dtype=torch.float32, device=flat.flat.device)
        self._lr_host = None
        self.grad_scale = 1.0
        self.steps = 0

    def _join(self):
        """Weight gradients may still be in flight on the wgrad side stream."""
        if self.flat.grad.is_cuda:
            from ..ops import streams
            streams.join(self.flat.grad.device)

    def _sync_lr(self):
        if self.lr_t.is_cuda and torch.cuda.is_current_stream_capturing():
            return   # the host-side lr write must stay outside a captured graph
        lr = float(self.param_groups[0]["lr"])
        if lr != self._lr_host:
            self.lr_t.fill_(lr)
            self._lr_host = lr

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()
        # a new step starts: slices an abandoned step updated early must not be skipped by
        # the next step()
        if hasattr(self, "_applied"):
            self._applied = []

    def state_dict(self) -> Dict:
        """torch.optim.SGD-format state dict (per-parameter momentum_buffer)."""
        st = {}
        for i, p in enumerate(self.flat.params):
            st[i] = {"momentum_buffer": self.flat._view(self.buf, i).detach().clone().contiguous()}
        g = {k: v for k, v in self.param_groups[0].items() if k != "params"}
        g["params"] = list(range(len(self.flat.params)))
        return {"state": st, "param_groups": [g]}

    def load_state_dict(self, sd: Dict):
        st = sd.get("state", {})
        for i, p in enumerate(self.flat.params):
            if i in st and "momentum_buffer" in st[i] and st[i]["momentum_buffer"] is not None:
                self.flat._view(self.buf, i).copy_(st[i]["momentum_buffer"])
        if sd.get("param_groups"):
            for k, v in sd["param_groups"][0].items():
                if k != "params":
                    self.param_groups[0][k] = v


class FusedSGD(_FlatOptimizer):
    """torch.optim.SGD(momentum, weight_decay, dampening=0) over the flat buffer."""

    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                 nesterov: bool = False, backend: str = "auto"):
        super().__init__(flat, lr, momentum, weight_decay)
        self.nesterov = nesterov
        self.native = backend != "torch" and flat.flat.is_cuda and _ext.available()
        self._applied = []      # [start, end) slices updated early this step (apply_range)
        import os
        self._early_blocks = int(os.environ.get("SDX_EARLY_STEP_BLOCKS", "0") or 0)

    @torch.no_grad()
    def apply_range(self, start: int, end: int):
        """Update the flat slice [start, end) now, on the current stream (the bucket reducer's
        early step: its gradients are final); :meth:`step` then skips it. Native path only."""
        f = self.flat
        _ext.require().sgd_step(f.flat[start:end], f.grad[start:end], self.buf[start:end], self.lr_t, self.momentum,
                                self.weight_decay, self.grad_scale, self.nesterov, self._early_blocks)
        self._applied.append((start, end))

    @torch.no_grad()
    def step(self):
        self._sync_lr()
        self._join()
        f = self.flat
        if self.native:
            m = _ext.require()
            # the slices no early apply_range covered (all of it without a bucket reducer)
            pos, n = 0, f.flat.numel()
            for a, b in sorted(self._applied) + [(n, n)]:
                if a > pos:
                    m.sgd_step(f.flat[pos:a], f.grad[pos:a], self.buf[pos:a], self.lr_t, self.momentum,
                               self.weight_decay, self.grad_scale, self.nesterov)
                pos = max(pos, b)
            self._applied = []
        else:
            d = f.grad * self.grad_scale
            if self.weight_decay:
                d.add_(f.flat, alpha=self.weight_decay)
            self.buf.mul_(self.momentum).add_(d)
            step = d.add(self.buf, alpha=self.momentum) if self.nesterov else self.buf
            f.flat.sub_(step * self.lr_t)
        self.steps += 1


class FusedLARS(_FlatOptimizer):
    """LARS (You et al.) with BN/bias excluded from adaptation and weight decay."""

    def __init__(self, flat: FlatParams, lr: float, momentum: float = 0.9, weight_decay: float = 0.0,
                 eta: float = 0.001, backend: str = "auto"):
        super().__init__(flat, lr, momentum, weight_decay)
        self.eta = eta
        offs, adapt = flat.segment_table()
        dev = flat.flat.device
        self.seg_off = torch.tensor(offs, dtype=torch.int64, device=dev)
        self.adapt = torch.tensor(adapt, dtype=torch.int32, device=dev)
        self.norms = torch.zeros(2 * len(offs), dtype=torch.float32, device=dev)
        self.native = backend != "torch" and flat.flat.is_cuda and _ext.available()

    @torch.no_grad()
    def step(self):
        self._sync_lr()
        self._join()
        f = self.flat
        if self.native:
            _ext.require().lars_step(f.flat, f.grad, self.buf, self.seg_off, self.adapt, self.lr_t, self.momentum,
                                     self.weight_decay, self.grad_scale, self.eta, self.norms)
        else:
            for i, p in enumerate(f.params):
                pv = f._view(f.flat, i)
                g = f._view(f.grad, i) * self.grad_scale
                b = f._view(self.buf, i)
                if p.dim() > 1:
                    d = g + self.weight_decay * pv
                    pn, dn = pv.norm(), d.norm()
                    trust = torch.where((pn > 0) & (dn > 0), self.eta * pn / dn, torch.ones_like(pn))
                else:
                    d = g
                    trust = torch.ones((), device=pv.device)
                b.mul_(self.momentum).add_(self.lr_t * trust * d)
                pv.sub_(b)
        self.steps += 1


def build_optimizer(name: str, flat: FlatParams, lr: float, momentum: float, weight_decay: float,
                    backend: str = "auto"):
    if name == "sgd":
        return FusedSGD(flat, lr, momentum, weight_decay, backend=backend)
    if name == "lars":
        return FusedLARS(flat, lr, momentum, weight_decay, backend=backend)
    raise ValueError(name)
