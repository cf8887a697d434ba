"""One-shot small-message all-reduce over xGMI peer memory.

SyncBN issues one fp64 all-reduce of ``[2, C]`` statistics per BatchNorm layer in the
forward pass and one of ``[2|3, C]`` sums in the backward pass (≈100 per ResNet-50 step,
≤16 KiB each), all on the critical path. A ring collective pays 2(W−1) link hops per
call; here every rank writes its payload once into every peer's IPC-mapped arena and
publishes an epoch flag, so a call costs one xGMI write + one flag round trip
(csrc/kernels/xgmi.hip). Arenas are exchanged once at start-up through the process group.

Requires all ranks on ONE node (``LOCAL_WORLD_SIZE == WORLD_SIZE``) and ≤ 8 of them; the
engine falls back to the RCCL all-reduce otherwise, or if the start-up self-check fails.
Enabled with ``--syncbn_comm xgmi``.
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

    def __init__(self, group=None, cap: int = 8192, timeout_s: float = 600.0):
        from . import comm
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("process group not initialised")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.m = _ext.require()
        self.cap = cap
        self.id = None
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

        ok, err = comm.negotiate([check_topology, create, exchange, open_peers, self._self_check], self.close, group)
        if not ok:
            raise RuntimeError(f"one-shot xGMI all-reduce unavailable ({err if err is not None else 'on a peer rank'})")

    def _self_check(self):
        dev = torch.device("cuda", torch.cuda.current_device())
        x = torch.arange(16, dtype=torch.float64, device=dev) + 100.0 * self.rank
        out = self.all_reduce(x)
        torch.cuda.synchronize()
        err = self.m.xgmi_error(self.id)
        exp = torch.arange(16, dtype=torch.float64, device=dev) * self.world + 100.0 * sum(range(self.world))
        if not (err == 0 and torch.equal(out, exp)):
            raise RuntimeError(f"one-shot xGMI all-reduce self-check failed (err={err})")

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        """Sum over ranks of a small fp64 tensor (returns a new tensor)."""
        if x.numel() > self.cap:
            raise ValueError("message larger than the arena slot")
        return self.m.xgmi_allreduce(self.id, x.contiguous()).view_as(x)

    def all_reduce_(self, x: torch.Tensor) -> torch.Tensor:
        x.copy_(self.all_reduce(x))
        return x

    def close(self):
        if getattr(self, "id", None) is not None:
            self.m.xgmi_destroy(self.id)
            self.id = None


def emulate(inputs: torch.Tensor, iters: int = 4) -> torch.Tensor:
    """Run the one-shot protocol for W virtual ranks on one GPU (tests)."""
    return _ext.require().xgmi_emulate(inputs.contiguous(), iters)
