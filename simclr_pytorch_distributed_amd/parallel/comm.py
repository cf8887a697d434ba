"""Process-group bootstrap and differentiable collectives.

Bootstrap (replaces main_supcon.py:357-364): ranks come from the launcher environment
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``), rendezvous is ``env://`` against
``MASTER_ADDR``/``MASTER_PORT``, the backend is RCCL (``"nccl"``) on GPUs and gloo on
CPU. A collective timeout is always set so a dead peer produces an error
instead of a hang.

Differentiable collectives:

* :func:`all_gather_with_grad` — forward all-gather of a per-rank block; backward is a
  reduce-scatter (sum) of the gathered gradient back to its owners. This is what makes
  the cross-GPU negatives of the contrastive loss (reference main_supcon.py:268-281,
  which only supported exactly 2 ranks and dropped the gradients of gathered copies)
  exact for any world size.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized()


class EmulatedGroup:
    """W identical virtual ranks on ONE GPU standing in for a SyncBN process group
    (``SDX_SYNCBN_EMU=W``; tools/syncbn_latency.py, bench at world 1). Registered with an
    emulated native communicator (comm_ops.cpp: EMU = reduce -> x·W -> finalize, or XEMU =
    the fused xGMI exchange through W device-memory arenas), every BN of the native
    executor runs its full cross-rank kernel sequence while the statistics stay exactly the
    single-process ones — so the step time shows the SyncBN cost minus the xGMI link
    latency, on the one-GPU box."""

    def __init__(self, world: int):
        self.world = int(world)


def group_size(group) -> int:
    """Ranks of a SyncBN group (None: 1; an :class:`EmulatedGroup`: its virtual ranks)."""
    if group is None:
        return 1
    if isinstance(group, EmulatedGroup):
        return group.world
    return dist.get_world_size(group)


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def backend() -> Optional[str]:
    return dist.get_backend() if is_dist() else None


def init_distributed(backend_name: str = "auto", timeout_s: float = 600.0, device: Optional[torch.device] = None):
    """Initialise the default process group if the launcher started >1 rank.

    Returns (rank, local_rank, world_size, device).
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rnk = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available()
    if device is None:
        # more local ranks than visible GPUs (a multi-rank rehearsal on a 1-GPU box):
        # ranks share devices round-robin instead of failing on a missing ordinal
        device = torch.device(f"cuda:{local % max(torch.cuda.device_count(), 1)}") if use_cuda \
            else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1 and not is_dist():
        if backend_name == "auto":
            backend_name = "nccl" if device.type == "cuda" else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # SDX_INIT_METHOD (e.g. file:///tmp/rdv): a port-free rendezvous for tests that
        # start ranks on a shared box, where a probed free port can be taken before use
        init = os.environ.get("SDX_INIT_METHOD", "env://")
        kw = dict(backend=backend_name, init_method=init, world_size=world, rank=rnk,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend_name == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rnk, local, world, device


def barrier():
    if is_dist():
        if backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def _supports_reduce_scatter() -> bool:
    return backend() == "nccl"


def all_gather_tensor(x: torch.Tensor) -> torch.Tensor:
    """Gather equal-sized blocks along dim 0 (no autograd)."""
    w = world_size()
    if w == 1:
        return x
    x = x.contiguous()
    out = torch.empty((w * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x)
    return out


def reduce_scatter_tensor(x: torch.Tensor) -> torch.Tensor:
    """Sum over ranks, then return this rank's dim-0 block (no autograd)."""
    w = world_size()
    if w == 1:
        return x
    x = x.contiguous()
    n = x.shape[0] // w
    if _supports_reduce_scatter():
        out = torch.empty((n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.reduce_scatter_tensor(out, x)
        return out
    y = x.clone()
    dist.all_reduce(y)
    r = rank()
    return y[r * n:(r + 1) * n].contiguous()


class _AllGatherGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return all_gather_tensor(x)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_tensor(g)


def all_gather_with_grad(x: torch.Tensor) -> torch.Tensor:
    if world_size() == 1:
        return x
    return _AllGatherGrad.apply(x)


_small = {}


def set_small_allreduce(group, impl) -> None:
    """Route :func:`small_all_reduce_` for ``group`` (None = WORLD) through ``impl``
    (e.g. :class:`parallel.xgmi.OneShotAllReduce`); ``impl=None`` restores RCCL/gloo."""
    key = id(group) if group is not None else None
    if impl is None:
        _small.pop(key, None)
    else:
        _small[key] = impl


_native = {}


def _key(group):
    return None if group is None or group is dist.group.WORLD else id(group)


def set_native_small_comm(group, handle: int) -> None:
    """Register a native small-communicator handle (csrc/bindings/comm_ops.cpp) for
    ``group`` (None = WORLD). The native block executor then issues the SyncBN
    all-reduces itself, in place on the compute stream; ``handle=0`` unregisters."""
    if handle:
        _native[_key(group)] = int(handle)
    else:
        _native.pop(_key(group), None)


def native_small_comm(group) -> int:
    """Handle for ``group`` (0 = none registered: use the Python collective path)."""
    return _native.get(_key(group), 0)


_gather = {}


def set_native_gather_comm(group, handle: int) -> None:
    """Register a native RCCL (or emulated) communicator that carries the contrastive
    loss's embedding all-gather / reduce-scatter for ``group``;
    ``handle=0`` unregisters (c10d path)."""
    if handle:
        _gather[_key(group)] = int(handle)
    else:
        _gather.pop(_key(group), None)


def native_gather_comm(group=None) -> int:
    return _gather.get(_key(group), 0)


def _agree_device(group=None) -> torch.device:
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def agree(ok: bool, group=None) -> bool:
    """True on every rank iff ``ok`` is true on every rank (one MIN all-reduce)."""
    if not is_dist():
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_agree_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def agree_fastest(names, times, eligible=None, group=None):
    """All ranks pick the same option from per-rank timings: ``times[i]`` (this rank's
    measurement of ``names[i]``) is MAX-reduced over the ranks — an option is as slow as its
    slowest rank — and every rank takes the argmin over ``eligible`` indices (default all) of
    the SAME reduced vector (ties: the first). Returns (name, reduced times)."""
    t = torch.tensor([float(v) for v in times], dtype=torch.float64, device=_agree_device(group)
                     if is_dist() else torch.device("cpu"))
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    red = t.tolist()
    idx = list(range(len(names))) if eligible is None else list(eligible)
    return names[min(idx, key=lambda i: (red[i], i))], red


def negotiate(steps, cleanup, group=None):
    """Run a multi-step set-up in which ranks must stay in lock-step.

    ``steps``: callables run in order on every rank. A step that runs a collective must
    be reached by all ranks or by none, so after EACH step the ranks agree (MIN
    all-reduce) that it succeeded everywhere before any rank starts the next one. If a
    step failed on any rank, every rank calls ``cleanup()`` (which must undo whatever
    part of the set-up this rank completed) and the function returns ``(False, err)``
    with this rank's own error (None where it succeeded) — all ranks together.
    """
    err = None
    for st in steps:
        try:
            st()
        except Exception as e:  # noqa: BLE001
            err = e
        if not agree(err is None, group):
            try:
                cleanup()
            except Exception:  # noqa: BLE001
                pass
            return False, err
    return True, None


def create_rccl_small_comm(group=None, timeout_s: float = 600.0) -> int:
    """A dedicated RCCL communicator over ``group``'s ranks for SyncBN statistics, or 0
    (on every rank together) if it cannot be set up anywhere.

    Rank 0 draws an ``ncclUniqueId`` and broadcasts it through the process group
    (the TCP/env rendezvous only carries this id); every rank then joins
    with a non-blocking ``ncclCommInitRankConfig`` polled against ``timeout_s`` and runs a
    self-check all-reduce. The ranks agree after every step (:func:`negotiate`), so a
    failure on one rank never leaves the others inside a mismatched collective; handles
    created before a failure are aborted locally. Kept apart from torch's communicators,
    so the gradient buckets on the reducer's comm stream never queue in front of a BN
    statistic (ordering argument: csrc/bindings/comm_ops.cpp).
    """
    from ..ops import _ext
    m = _ext.require()
    w, r = dist.get_world_size(group), dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    st = {"uid": torch.zeros(128, dtype=torch.uint8), "h": 0}

    def draw():
        if r == 0:
            st["uid"] = m.rccl_unique_id()

    def share():
        t = st["uid"].to(dev) if dist.get_backend(group) == "nccl" else st["uid"]
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        st["uid"] = t.cpu()

    def join():
        st["h"] = m.rccl_comm_init(st["uid"], w, r, float(min(timeout_s, 300.0)))

    def check():
        probe = torch.ones(4, dtype=torch.float64, device=dev)
        m.small_all_reduce_(st["h"], probe)
        if float(probe[0].item()) != float(w):
            raise RuntimeError(f"RCCL small communicator self-check failed ({probe[0].item()} != {w})")
        # rank-major all-gather + reduce-scatter (the contrastive loss's embedding exchange)
        g = m.small_all_gather(st["h"], torch.full((2, 8), float(r), device=dev))
        want = torch.arange(w, device=dev, dtype=torch.float32).repeat_interleave(2)[:, None].expand(-1, 8)
        if not torch.equal(g, want):
            raise RuntimeError("RCCL small communicator all-gather self-check failed")
        rs = m.small_reduce_scatter(st["h"], torch.ones(2 * w, 8, device=dev))
        if not torch.equal(rs, torch.full((2, 8), float(w), device=dev)):
            raise RuntimeError("RCCL small communicator reduce-scatter self-check failed")

    def cleanup():
        if st["h"]:
            m.small_comm_abort(st["h"])
            st["h"] = 0

    ok, err = negotiate([draw, share, join, check], cleanup, group)
    if not ok:
        import logging
        logging.warning(f"dedicated RCCL communicator unavailable ({err if err is not None else 'on a peer rank'})")
        return 0
    return st["h"]


def small_all_reduce_(x: torch.Tensor, group=None) -> torch.Tensor:
    """In-place sum of a small, latency-bound tensor (SyncBN statistics)."""
    h = _native.get(_key(group), 0)
    if h and x.is_cuda and x.is_contiguous() and x.dtype == torch.float64:
        from ..ops import _ext
        _ext.require().small_all_reduce_(h, x)
        return x
    impl = _small.get(id(group) if group is not None else None)
    if impl is None and group is dist.group.WORLD:
        impl = _small.get(None)
    if impl is not None and x.is_cuda and x.dtype == torch.float64:
        return impl.all_reduce_(x)
    dist.all_reduce(x, group=group)
    return x


def all_reduce_sum_(x: torch.Tensor) -> torch.Tensor:
    if world_size() > 1:
        dist.all_reduce(x)
    return x
