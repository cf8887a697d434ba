"""Gradient sinks: fused backward kernels write parameter gradients straight into
``param.grad`` (a view of the flat gradient buffer) instead of returning new tensors
through autograd's AccumulateGrad (which costs an allocation and an extra add pass per
parameter). Writers always ACCUMULATE (the buffer is zeroed by ``zero_grad``), so
gradient accumulation over micro-batches stays correct.

Listeners (the data-parallel bucket reducer) are told when a parameter's gradient is
final for this backward pass, exactly as autograd's post-accumulate hooks would.
"""
from __future__ import annotations

from typing import Callable, Iterable, List

import torch

_listeners: List[Callable[[torch.nn.Parameter], None]] = []


def add_listener(fn: Callable[[torch.nn.Parameter], None]):
    _listeners.append(fn)
    return fn


def remove_listener(fn):
    if fn in _listeners:
        _listeners.remove(fn)


def target(p: torch.nn.Parameter) -> torch.Tensor:
    """The tensor to accumulate ``p``'s gradient into (allocated zero if absent)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.preserve_format)
    return p.grad


def notify(params: Iterable[torch.nn.Parameter]):
    if not _listeners:
        return
    for p in params:
        for fn in _listeners:
            fn(p)
