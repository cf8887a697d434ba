"""Side HIP stream for weight-gradient GEMMs.

In a residual block's backward the data-gradient chain (BN backward → dgrad → BN
backward → ...) is the critical path; each conv's weight gradient only feeds the
optimizer. The fused block backward (ops/block.py) therefore issues every wgrad on a
side stream that forks from the compute stream (event) and is joined once at the end of
backward (:func:`join`), so wgrads and their split-K reductions fill the bubbles of the
latency-bound BN/reduction kernels. Inside a captured hipGraph the fork/join become
parallel graph branches.

Tensors the side stream reads are kept alive in a stash until the join (instead of
``record_stream``): after the join the compute stream is ordered behind every side-stream
kernel, so the stashed blocks return to the caching allocator reusable at once, in program
order. With ``record_stream`` each block stayed unusable until a side-stream event had
completed; since the host runs ahead of the GPU the allocator kept mapping new segments
(35 GiB reserved for a 7 GiB peak, and a hipMalloc every few steps).
"""
from __future__ import annotations

import os

import torch

_side = {}
ENABLED = os.environ.get("SDX_WGRAD_STREAM", "1") != "0"


def side(device: torch.device) -> torch.cuda.Stream:
    key = device.index if device.index is not None else torch.cuda.current_device()
    s = _side.get(key)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _side[key] = s
    return s


_stash = []


def stash(*tensors):
    """Keep ``tensors`` alive until the next :func:`join` (they are read by side-stream work)."""
    _stash.extend(t for t in tensors if t is not None)


class SideWork:
    """``with SideWork(t1, t2, ...):`` runs the body on the side stream after all work
    queued so far on the current stream; listed tensors are protected for that stream."""

    def __init__(self, *tensors):
        self.tensors = tensors
        self.active = ENABLED and tensors[0].is_cuda
        self._ctx = None

    def __enter__(self):
        if not self.active:
            return self
        dev = self.tensors[0].device
        main = torch.cuda.current_stream(dev)
        s = side(dev)
        s.wait_event(main.record_event())
        stash(*self.tensors)
        self._ctx = torch.cuda.stream(s)
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self._ctx is not None:
            self._ctx.__exit__(*exc)
        return False


def join(device: torch.device):
    """Make the current stream wait for everything issued on the side stream."""
    if ENABLED and device.type == "cuda":
        key = device.index if device.index is not None else torch.cuda.current_device()
        s = _side.get(key)
        if s is not None:
            torch.cuda.current_stream(device).wait_stream(s)
        release()


def release():
    """Drop the stash (Python and native executor); only valid after the join."""
    _stash.clear()
    from . import _ext
    if _ext.available():
        _ext.require().side_stash_release()
