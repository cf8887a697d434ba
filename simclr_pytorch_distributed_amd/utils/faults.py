"""Failure detection and fault injection (the reference has neither: an NCCL
error or a dead peer hangs or kills the job, main_supcon.py:359-364).

* Every process group is created with a collective timeout (``--comm_timeout``), so a
  peer that dies or stalls surfaces as an exception instead of a hang.
* :func:`guarded_main` runs an entry point and turns a collective failure into ONE clear
  log line naming the rank, a best-effort process-group teardown and exit status 3.
* :func:`maybe_inject` is a deterministic fault-injection hook for drills and tests,
  configured by ``SDX_FAULT_INJECT="rank=R,step=S[,mode=exit|raise|hang]"``: the given rank
  exits (status 17), raises, or sleeps at the given global step.
"""
from __future__ import annotations

import logging
import os
import sys
import time
from typing import Callable, Optional

FAULT_EXIT_CODE = 17
COLLECTIVE_FAILURE_EXIT_CODE = 3


class InjectedFault(RuntimeError):
    pass


def _parse(spec: str) -> dict:
    out = {}
    for part in spec.split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip()] = v.strip()
    return out


_SPEC: Optional[dict] = None


def fault_spec() -> dict:
    global _SPEC
    if _SPEC is None:
        s = os.environ.get("SDX_FAULT_INJECT", "")
        _SPEC = _parse(s) if s else {}
    return _SPEC


def maybe_inject(rank: int, step: int) -> None:
    spec = fault_spec()
    if not spec:
        return
    if int(spec.get("rank", -1)) != rank or int(spec.get("step", -1)) != step:
        return
    mode = spec.get("mode", "exit")
    logging.error(f"[fault-inject] rank {rank} step {step}: {mode}")
    if mode == "raise":
        raise InjectedFault(f"injected fault on rank {rank} at step {step}")
    if mode == "hang":
        time.sleep(float(spec.get("seconds", "3600")))
        return
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(FAULT_EXIT_CODE)


def is_collective_failure(e: BaseException) -> bool:
    name = type(e).__name__
    msg = str(e).lower()
    keys = ("connection", "timed out", "timeout", "peer", "nccl", "rccl", "gloo", "closed", "broken pipe",
            "process group", "watchdog")
    return name in ("DistBackendError", "DistNetworkError", "DistStoreError") or any(k in msg for k in keys)


def guarded_main(fn: Callable[[], object]) -> object:
    """Run ``fn``; a collective failure becomes one clear error line and exit code 3."""
    try:
        return fn()
    except InjectedFault:
        raise
    except Exception as e:  # noqa: BLE001
        if not is_collective_failure(e):
            raise
        import torch.distributed as dist
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else int(os.environ.get("RANK", 0))
        msg = (f"rank {rank}: collective failure (a peer rank died, stalled past --comm_timeout, or the "
               f"network failed): {type(e).__name__}: {str(e).splitlines()[0] if str(e) else ''}")
        logging.error(msg)
        print(msg, file=sys.stderr, flush=True)
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass
        sys.exit(COLLECTIVE_FAILURE_EXIT_CODE)
