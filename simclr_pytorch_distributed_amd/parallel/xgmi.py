"""One-shot small-message exchange over xGMI peer memory — the default
SyncBN transport of the native executor when every rank is on one node.

SyncBN needs one fp64 sum of ``[2, C]`` statistics per BatchNorm layer in the forward pass
and one of ``[2|3, C]`` sums in the backward pass (≈106 per ResNet-50 step, ≤24 KiB each;
reference: main_supcon.py:222-224 → torch SyncBatchNorm), all on the critical path. A ring
collective pays 2(W−1) link hops per call; here every rank writes its payload once into
every peer's IPC-mapped arena and publishes an epoch flag, so a call costs one xGMI write
+ one flag round trip. Arenas are exchanged once at start-up through the process group.

Two kernels use the arena:

* the FUSED path (default): the BN statistics' column reduction itself (csrc/kernels/bn.hip
  ``col_reduce`` with an ``XgmiCol``) stores each 64-channel group's sums into the peers'
  arenas, waits for theirs and runs the finalize / backward-coefficient epilogue on the
  global sums — reduce + all-reduce + finalize in ONE launch per BN;
* ``all_reduce``: the stand-alone one-shot kernel (csrc/kernels/xgmi.hip) for any small fp64
  tensor (``SDX_SYNCBN_FUSED=0`` routes the executor through it).

Requires all ranks on ONE node (``LOCAL_WORLD_SIZE == WORLD_SIZE``) and ≤ 8 of them; the
engine falls back to a dedicated RCCL communicator otherwise, or if a start-up self-check
(stand-alone and fused exchange against known sums) fails on any rank.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _ext


class OneShotAllReduce:
    """Set-up runs as :func:`parallel.comm.negotiate` steps (create the arena, exchange
    IPC handles, map the peers, self-check), with the ranks agreeing after each one: a
    rank that fails to allocate or map raises on EVERY rank (after each rank destroyed
    its own arena), never only on itself while its peers wait in a collective."""

    CHECK_TIMEOUT_S = 30.0   # deadline of each start-up self-check kernel

    def __init__(self, group=None, cap: int = 12288, timeout_s: float = 600.0):
        from . import comm
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("process group not initialised")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.m = _ext.require()
        self.cap = cap
        self.id = None
        self.handle = 0          # native small-communicator wrapping the arena (comm_ops.cpp)
        st = {}

        def check_topology():
            if self.world > 8:
                raise RuntimeError("one-shot xGMI all-reduce supports at most 8 ranks")
            lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world)))
            if lws != self.world:
                raise RuntimeError("one-shot xGMI all-reduce needs every rank on one node")

        def create():
            self.id = self.m.xgmi_create(self.rank, self.world, cap, float(timeout_s))
            st["mine"] = bytes(self.m.xgmi_handle(self.id).numpy().tobytes())

        def exchange():
            allh = [None] * self.world
            dist.all_gather_object(allh, st["mine"], group=group)
            st["h"] = torch.frombuffer(bytearray(b"".join(allh)), dtype=torch.uint8).view(self.world, 64).clone()

        def open_peers():
            self.m.xgmi_open(self.id, st["h"])

        def wrap():
            self.handle = self.m.xgmi_small_comm(self.id, self.rank, float(timeout_s))

        # the checks run on the bare arena with a short deadline: a peer that never answers
        # fails the check on every rank (-> RCCL fallback); only a checked arena is wrapped
        # (and so watched by the communicator watchdog)
        ok, err = comm.negotiate([check_topology, create, exchange, open_peers, self._self_check, self._fused_check,
                                  wrap], self.close, group)
        if not ok:
            raise RuntimeError(f"one-shot xGMI all-reduce unavailable ({err if err is not None else 'on a peer rank'})")

    def _self_check(self):
        dev = torch.device("cuda", torch.cuda.current_device())
        x = torch.arange(16, dtype=torch.float64, device=dev) + 100.0 * self.rank
        out = self.m.xgmi_allreduce(self.id, x, self.CHECK_TIMEOUT_S)
        torch.cuda.synchronize()
        err = self.m.xgmi_error(self.id)
        exp = torch.arange(16, dtype=torch.float64, device=dev) * self.world + 100.0 * sum(range(self.world))
        if not (err == 0 and torch.equal(out, exp)):
            raise RuntimeError(f"one-shot xGMI all-reduce self-check failed (err={err})")

    def _fused_check(self):
        """The fused SyncBN exchange (column reduction + exchange in one launch) on slabs
        with rank-dependent values and the BN shapes' extremes: C = 64 (one group) and
        C = 2048 with 3 sums (32 groups), rows 1 and 300."""
        dev = torch.device("cuda", torch.cuda.current_device())
        for rows, ns, C in ((1, 2, 64), (300, 3, 2048), (37, 2, 200)):
            base = torch.arange(rows * ns * C, dtype=torch.float64, device=dev).remainder(97).view(rows, ns, C)
            slab = (base + self.rank).float()
            got = self.m.xgmi_exchange_sums(self.id, slab.contiguous(), self.CHECK_TIMEOUT_S)
            exp = base.sum(0) * self.world + rows * sum(range(self.world))
            torch.cuda.synchronize()
            if self.m.xgmi_error(self.id) != 0 or not torch.allclose(got, exp, rtol=0, atol=1e-6):
                raise RuntimeError(f"fused xGMI SyncBN exchange self-check failed (rows {rows}, C {C})")

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        """Sum over ranks of a small fp64 tensor (returns a new tensor)."""
        if x.numel() > self.cap:
            raise ValueError("message larger than the arena slot")
        return self.m.xgmi_allreduce(self.id, x.contiguous()).view_as(x)

    def all_reduce_(self, x: torch.Tensor) -> torch.Tensor:
        x.copy_(self.all_reduce(x))
        return x

    def close(self):
        # the wrapping communicator first: the watchdog must stop sweeping the arena before
        # it is freed
        if getattr(self, "handle", 0):
            self.m.small_comm_destroy(self.handle)
            self.handle = 0
        if getattr(self, "id", None) is not None:
            self.m.xgmi_destroy(self.id)
            self.id = None


def emulate(inputs: torch.Tensor, iters: int = 4) -> torch.Tensor:
    """Run the one-shot protocol for W virtual ranks on one GPU (tests)."""
    return _ext.require().xgmi_emulate(inputs.contiguous(), iters)
