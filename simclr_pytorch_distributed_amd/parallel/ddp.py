"""Bucketed data-parallel gradient all-reduce, overlapped with backward.

Replaces ``torch.nn.parallel.DistributedDataParallel`` (main_supcon.py:230-234) with a
reducer built on the flat gradient buffer of :class:`optim.flat.FlatParams`:

* buckets are contiguous slices of the flat gradient (segments are laid out in backward
  order), so each bucket is all-reduced *in place* — no copy into bucket buffers;
* a post-accumulate-grad hook counts ready parameters; when a bucket is complete the
  compute stream records an event, the dedicated communication stream waits on it and
  issues the RCCL all-reduce (SUM) there, so the collective runs over xGMI while
  backward keeps computing earlier layers;
* averaging is not a separate pass: the optimizer kernel applies ``1/W`` (grad_scale)
  while it streams the gradients (``--grad_semantics exact`` keeps the sum);
* bucket size defaults to 24 MiB (ResNet-50 + head: 112 MB of fp32 gradients -> 5
  buckets). The constraint is overlap, not per-call latency: a bucket can only launch
  when its last gradient exists, and the last bucket (layer 2/1 + stem) is exposed after
  backward. With 64 MiB buckets the second (~48 MB) launched only at finish(); at 24 MiB
  the layer-3 gradients go out while layer 2/1 are still in backward, leaving a few MB
  for the tail. Per collective an 8-rank ring over xGMI moves 2(W-1)/W of the bucket
  through one ~153 GB/s link per step, i.e. ≈0.3 ms for 24 MiB — well under the
  backward time that follows each launch, and ≫ the ~20-40 µs fixed cost of a launch;
* parameters/buffers are broadcast from rank 0 once at construction (one collective on
  the flat buffer); the per-forward BN buffer broadcast of DDP is dropped;
* ``early_step(start, end)`` (optional, e.g. :meth:`optim.flat.FusedSGD.apply_range`): the
  optimizer update of a bucket's slice, issued on the communication stream right after
  the bucket's collective (or, with one rank, as soon as its gradients are final), so the
  elementwise update of the deeper layers runs while backward is still computing the
  shallow ones and only the last bucket's update is left after backward (the whole-buffer
  SGD pass was ~90 us at the end of the ResNet-50 step). Used with one rank as well;
* ``compress='bf16'`` (``--grad_compress bf16``): each bucket is all-reduced as a bf16 copy
  (half the bytes over the per-link-bound xGMI ring; the sum is rounded to bf16 — the
  reference DDP reduces fp32, so this is opt-in) and written back into the fp32 buffer.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from . import comm


class GradBucketReducer:
    def __init__(self, flat, bucket_mb: Optional[float] = None, group=None, enabled: Optional[bool] = None,
                 broadcast_init: bool = True, early_step=None, compress: str = "none"):
        if bucket_mb is None:
            import os
            bucket_mb = float(os.environ.get("SDX_BUCKET_MB", "24"))
        self.flat = flat
        self.group = group
        self.world = comm.world_size() if group is None else dist.get_world_size(group)
        self.enabled = (self.world > 1) if enabled is None else enabled   # all-reduce the buckets
        self.early_step = early_step
        if compress not in ("none", "bf16"):
            raise ValueError(f"compress must be 'none' or 'bf16', got {compress!r}")
        self.compress = compress
        self.active = self.enabled or early_step is not None            # track bucket completion
        cap = int(bucket_mb * (1 << 20) / 4)
        # buckets in backward (= flat buffer) order
        self.buckets: List[dict] = []
        cur = None
        for i in flat.order:
            start = flat.offsets[i]
            end = start + (flat.params[i].numel() + 4095) // 4096 * 4096
            if cur is None or (end - cur["start"]) > cap and cur["params"]:
                cur = {"start": start, "end": end, "params": [], "ready": 0, "work": None, "launched": False,
                       "cbuf": None, "idx": len(self.buckets)}
                self.buckets.append(cur)
            cur["params"].append(i)
            cur["end"] = end
        self.bucket_of = {}
        for b_idx, b in enumerate(self.buckets):
            for i in b["params"]:
                self.bucket_of[i] = b_idx
        self.is_cuda = flat.grad.is_cuda
        self.comm_stream = torch.cuda.Stream(device=flat.grad.device) if (self.is_cuda and self.active) else None
        self._hooks = []
        self._index = {id(p): i for i, p in enumerate(flat.params)}
        # a parameter is counted once per backward: fused blocks notify through their gradient
        # sink AND autograd still runs the parameter's AccumulateGrad node (with a None grad),
        # which fires the post-accumulate hook a second time
        self._seen = [False] * len(flat.params)
        self._paused = False
        self._listener = None
        self.launch_log: List[int] = []     # bucket indices in launch order (tests, profiling)
        if self.active:
            for i, p in enumerate(flat.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            # fused native blocks write gradients into their sinks directly and notify here
            from ..ops import sinks
            self._listener = sinks.add_listener(self._on_sink)
        if self.enabled and broadcast_init:
            self.broadcast_parameters()

    def _on_sink(self, p):
        i = self._index.get(id(p))
        if i is not None:
            self._make_hook(i)(p)

    # ---- init ---------------------------------------------------------------------
    @torch.no_grad()
    def broadcast_parameters(self, buffers_of: Optional[torch.nn.Module] = None):
        if not self.enabled:
            return
        dist.broadcast(self.flat.flat, src=0, group=self.group)
        mod = buffers_of if buffers_of is not None else self.flat.model
        for b in mod.buffers():
            dist.broadcast(b, src=0, group=self.group)

    # ---- backward -----------------------------------------------------------------
    def _make_hook(self, i):
        def hook(_p):
            if self._paused or self._seen[i]:
                return
            self._seen[i] = True
            b = self.buckets[self.bucket_of[i]]
            b["ready"] += 1
            if b["ready"] == len(b["params"]):
                self._launch(b)
        return hook

    def _reduce(self, b, view):
        """Issue the bucket's collective (async); with bf16 compression on a bf16 copy."""
        if self.compress == "bf16":
            b["cbuf"] = view.to(torch.bfloat16)
            b["work"] = dist.all_reduce(b["cbuf"], group=self.group, async_op=True)
        else:
            b["work"] = dist.all_reduce(view, group=self.group, async_op=True)

    def _complete(self, b):
        """Order the current stream after the bucket's collective (and copy a compressed sum
        back into the fp32 buffer)."""
        if b["work"] is not None:
            b["work"].wait()
            b["work"] = None
        if b["cbuf"] is not None:
            self.flat.grad[b["start"]:b["end"]].copy_(b["cbuf"])
            b["cbuf"] = None

    def _launch(self, b):
        view = self.flat.grad[b["start"]:b["end"]]
        b["launched"] = True
        if self.comm_stream is not None:
            ev = torch.cuda.current_stream().record_event()
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                # fused blocks compute weight gradients on the wgrad side stream. The hook
                # fires right after the block that owns the bucket's last parameter issued
                # its wgrads, and the side stream is FIFO, so this wait ends with that
                # bucket's last wgrad — not behind wgrads of later (shallower) blocks.
                from ..ops import streams
                if streams.ENABLED:
                    self.comm_stream.wait_stream(streams.side(view.device))
                if self.enabled:
                    self._reduce(b, view)
                if self.early_step is not None:
                    self._complete(b)        # orders the comm stream after the collective
                    self.early_step(b["start"], b["end"])
            self.launch_log.append(b["idx"])
        else:
            if self.enabled:
                self._reduce(b, view)
            if self.early_step is not None:
                self._complete(b)
                self.early_step(b["start"], b["end"])
            self.launch_log.append(b["idx"])

    def no_sync(self):
        """Context: gradients produced inside only accumulate locally (no bucket launches),
        e.g. all but the last micro-batch of a gradient-cache step."""
        import contextlib

        @contextlib.contextmanager
        def _ctx():
            prev, self._paused = self._paused, True
            try:
                yield
            finally:
                self._paused = prev
        return _ctx()

    def finish(self):
        """Wait for all bucket reductions (launching any bucket whose params got no grad)."""
        if not self.active:
            return
        if self.is_cuda:
            from ..ops import streams
            streams.join(self.flat.grad.device)
        for b in self.buckets:
            if not b["launched"]:
                self._launch(b)
        for b in self.buckets:
            if self.comm_stream is not None and b["cbuf"] is not None:
                with torch.cuda.stream(self.comm_stream):
                    self._complete(b)
            else:
                self._complete(b)
            b["launched"] = False
            b["ready"] = 0
        self._seen = [False] * len(self._seen)
        if self.comm_stream is not None:
            torch.cuda.current_stream().wait_stream(self.comm_stream)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self._listener is not None:
            from ..ops import sinks
            sinks.remove_listener(self._listener)
            self._listener = None
