"""Loader for the in-tree gfx950 extension ``simclr_pytorch_distributed_amd._C``.

The extension is built by ``csrc/build.py`` (``__graft_entry__.build()``). If it is
missing or stale, :func:`ext` rebuilds it in-tree once (hipcc cross-compiles without a
GPU). A GPU run that asked for the native backend never silently falls back to torch
ops: :func:`require` raises if the extension cannot be loaded.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err = None


def _src_newer_than_so() -> bool:
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    so = os.path.join(root, "simclr_pytorch_distributed_amd", "_C.so")
    if not os.path.exists(so):
        return True
    t = os.path.getmtime(so)
    csrc = os.path.join(root, "csrc")
    if not os.path.isdir(csrc):
        return False
    for d, _, files in os.walk(csrc):
        for f in files:
            if f.endswith((".hip", ".cpp", ".h")) and os.path.getmtime(os.path.join(d, f)) > t:
                return True
    return False


def ext():
    """Return the extension module or None if it cannot be built/loaded."""
    global _mod, _err
    if _mod is not None or _err is not None:
        return _mod
    with _lock:
        if _mod is not None or _err is not None:
            return _mod
        try:
            if os.environ.get("SDX_AUTOBUILD", "1") != "0" and _src_newer_than_so():
                import sys
                root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
                sys.path.insert(0, os.path.join(root, "csrc"))
                try:
                    import build as _b  # csrc/build.py
                    _b.build()
                finally:
                    sys.path.pop(0)
            # SDX_CHECKED=1: the bounds-checked build (csrc/build.py --checked)
            # SDX_EXT_VARIANT=v: an experiment build (csrc/build.py --variant v)
            var = os.environ.get("SDX_EXT_VARIANT", "")
            name = "_C_checked" if os.environ.get("SDX_CHECKED", "0") == "1" else ("_C_" + var if var else "_C")
            _mod = importlib.import_module("simclr_pytorch_distributed_amd." + name)
        except Exception as e:  # noqa: BLE001
            _err = e
            _mod = None
    return _mod


def available() -> bool:
    return ext() is not None


def require():
    m = ext()
    if m is None:
        raise RuntimeError(f"native gfx950 extension unavailable: {_err!r}; run `python csrc/build.py`")
    return m
