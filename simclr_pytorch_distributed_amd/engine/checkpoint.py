"""Checkpoints compatible with the reference in both directions (util.py:87-96).

Layout written: ``{'opt', 'model', 'optimizer', 'epoch'}`` — ``model`` keys carry the
``module.`` prefix exactly as a DDP-wrapped reference model's ``state_dict()`` does
(322 keys for ResNet-50), tensors contiguous in NCHW layout; ``optimizer``
is a torch.optim.SGD state dict. ``opt`` is stored as a plain dict of JSON-like values
(no pickled ``argparse.Namespace`` / device tensors), so our own checkpoints load with
``torch.load(weights_only=True)``. Extra keys for true resume:
``sdx_state`` = {record_norm_mean, sampler epoch, rng states, global step}.

Loading (:func:`load_model_state`) accepts both prefixed and unprefixed keys (fixes the
reference's prefix mismatch). Reference-produced checkpoints contain a
pickled Namespace; they are loaded with ``weights_only=True`` plus an allow-list for
``argparse.Namespace`` — never with unrestricted unpickling.
"""
from __future__ import annotations

import argparse
import os
from typing import Any, Dict, Optional

import torch

PREFIX = "module."


def _plain(v: Any):
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    if isinstance(v, (list, tuple)):
        return [_plain(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _plain(x) for k, x in v.items()}
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().tolist() if v.numel() < 64 else None
    return str(v)


def opt_to_dict(opt) -> Dict[str, Any]:
    d = vars(opt) if isinstance(opt, argparse.Namespace) else dict(opt)
    return {k: _plain(v) for k, v in d.items()}


def model_state_with_prefix(model: torch.nn.Module, prefix: str = PREFIX) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in model.state_dict().items():
        out[prefix + k] = v.detach().clone().contiguous()
    return out


def save_model(model, optimizer, opt, epoch: int, save_file: str, extra: Optional[Dict] = None):
    print("==> Saving...")
    state = {
        "opt": opt_to_dict(opt),
        "model": model_state_with_prefix(model),
        "optimizer": optimizer.state_dict(),
        "epoch": int(epoch),
    }
    if extra:
        state["sdx_state"] = extra
    tmp = save_file + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, save_file)
    del state


def load_checkpoint(path: str, map_location="cpu") -> Dict:
    """Load without executing arbitrary pickled code (weights_only=True + allow-list)."""
    try:
        return torch.load(path, map_location=map_location, weights_only=True)
    except Exception:
        with torch.serialization.safe_globals([argparse.Namespace]):
            return torch.load(path, map_location=map_location, weights_only=True)


def strip_prefix(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {(k[len(PREFIX):] if k.startswith(PREFIX) else k): v for k, v in sd.items()}


def load_model_state(model: torch.nn.Module, sd: Dict[str, torch.Tensor], strict: bool = True):
    sd = strip_prefix(sd)
    own = model.state_dict()
    with torch.no_grad():
        missing = [k for k in own if k not in sd]
        unexpected = [k for k in sd if k not in own]
        if strict and (missing or unexpected):
            raise KeyError(f"state dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
        for k, v in sd.items():
            if k in own:
                own[k].copy_(v.to(own[k].device, own[k].dtype))
    return missing, unexpected
