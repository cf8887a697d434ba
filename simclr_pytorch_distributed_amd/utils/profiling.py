"""Tracing and per-phase timing (the reference has only wall-clock
``AverageMeter``s, main_supcon.py:248-254, 336-337).

* :func:`range_push` / :func:`range_pop` / :func:`mark` emit ROCTX ranges through
  ``libroctx64.so`` (ctypes, no torch dependency), so ``rocprofv3 --marker-trace`` shows
  the step phases next to the kernels. They are no-ops when the library is absent.
* :class:`PhaseTimer` brackets the phases of a training step (augment, forward, loss,
  backward, gradient-sync wait, optimizer) with HIP events recorded on the current
  stream. Elapsed times are read only when :meth:`PhaseTimer.summary` is called (at the
  print frequency), so timing adds no host synchronisation to the step.

Enabled with ``--profile`` on main_supcon.py / main_linear.py.
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os
from collections import OrderedDict, defaultdict
from typing import Dict, List, Optional, Tuple

import torch

_lib = None
_lib_tried = False


def _roctx():
    global _lib, _lib_tried
    if _lib_tried:
        return _lib
    _lib_tried = True
    names = ["libroctx64.so", "libroctx64.so.4"]
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for n in names:
        for cand in (os.path.join(rocm, "lib", n), n):
            try:
                lib = ctypes.CDLL(cand)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                return _lib
            except OSError:
                continue
    return None


def available() -> bool:
    return _roctx() is not None


def range_push(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def range_pop() -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def trace_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


class PhaseTimer:
    """Per-phase HIP-event timer for a training step.

    ``with timer.phase("fwd"): ...`` records a start/end event pair on the current
    stream (and a ROCTX range). Pairs are kept until :meth:`summary` converts them into
    mean milliseconds per step and frees them. Disabled timers cost nothing; phases are
    skipped automatically while a HIP graph is being captured.
    """

    def __init__(self, enabled: bool = False, device: Optional[torch.device] = None, roctx: bool = True):
        self.enabled = bool(enabled)
        self.cuda = device is not None and device.type == "cuda" and torch.cuda.is_available()
        self.roctx = roctx
        self._pending: Dict[str, List[Tuple[object, object]]] = defaultdict(list)
        self._host: Dict[str, List[float]] = defaultdict(list)
        self._order: "OrderedDict[str, None]" = OrderedDict()

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled or (self.cuda and torch.cuda.is_current_stream_capturing()):
            yield
            return
        self._order.setdefault(name, None)
        if self.roctx:
            range_push(name)
        if self.cuda:
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._pending[name].append((s, e))
                if self.roctx:
                    range_pop()
        else:
            import time
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._host[name].append((time.perf_counter() - t0) * 1e3)
                if self.roctx:
                    range_pop()

    def summary(self, reset: bool = True) -> "OrderedDict[str, float]":
        """Mean ms per occurrence of every phase since the last reset (synchronises on
        the recorded end events only)."""
        out: "OrderedDict[str, float]" = OrderedDict()
        for name in self._order:
            vals = list(self._host.get(name, []))
            for s, e in self._pending.get(name, []):
                e.synchronize()
                vals.append(s.elapsed_time(e))
            if vals:
                out[name] = sum(vals) / len(vals)
        if reset:
            self._pending.clear()
            self._host.clear()
        return out

    @staticmethod
    def format(summary: "OrderedDict[str, float]") -> str:
        return " ".join(f"{k} {v:.2f}" for k, v in summary.items())
