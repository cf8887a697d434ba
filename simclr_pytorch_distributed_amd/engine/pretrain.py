"""Contrastive pretraining engine (SimCLR / SupCon) — replaces main_supcon.py:155-406.

Per step (reference hot loop: main_supcon.py:253-349):

1. the rank's slice of the epoch permutation indexes the HBM-resident uint8 dataset and
   the fused GPU augmentation kernel writes both views (NHWC bf16) — no DataLoader
   workers, no H2D copy (reference: 8 CPU workers running PIL, main_supcon.py:200-207);
2. per-iteration warm-up lr (util.py:69-76) is written to the optimizer's device lr;
3. forward: native gfx950 encoder (or stock torch ops) + projection head;
4. loss: row-owned distributed SupCon/NT-Xent over globally gathered embeddings
   (losses/supcon.py) + the optional SEC / L2-reg feature-norm terms (main_supcon.py:295-317);
5. backward with bucketed gradient all-reduce overlapped on a comm stream
   (parallel/ddp.py), then one fused SGD/LARS kernel over the flat parameter buffer.

Logging keeps the reference's console format and TensorBoard tags; metric values stay on
device and are synchronised only every ``print_freq`` steps.
"""
from __future__ import annotations

import contextlib
import logging
import math
import os
import sys
import time
from typing import Optional

import torch
import torch.distributed as dist

from ..data.augment import AugConfig, augment, nhwc8_to_nchw
from ..data.augment import gpu_augment as augment_gpu
from ..data.datasets import build_dataset
from ..data.sampler import DistributedIndexSampler
from ..losses.supcon import DistributedContrastiveLoss
from ..models.executor import ModelRunner
from ..models.resnet import SupConResNet
from ..ops import _ext
from ..optim.flat import FlatParams, FusedSGD, build_optimizer
from ..optim.schedules import adjust_learning_rate, warmup_learning_rate
from ..parallel import comm

_ZERO_SIDE = os.environ.get("SDX_ZERO_SIDE", "1") != "0"
_NORM_SIDE = os.environ.get("SDX_NORM_SIDE", "1") != "0"
from ..parallel.ddp import GradBucketReducer
from ..utils.logging import setup_logging
from ..utils.meters import AverageMeter
from ..utils.faults import maybe_inject
from ..utils.profiling import PhaseTimer
from . import checkpoint as ckpt_mod


def resolve_backend(requested: str, device: torch.device, stem: str = "cifar") -> str:
    if requested == "torch":
        return "torch"
    native_ok = device.type == "cuda" and _ext.available()
    if requested == "native":
        if not native_ok:
            _ext.require()
            raise RuntimeError("native backend needs a GPU")
        return "native"
    return "native" if native_ok else "torch"


def _null():
    import contextlib
    return contextlib.nullcontext()


def step_seed(base: int, epoch: int, idx: int, rank: int) -> int:
    return (base * 1000003 + epoch * 100003 + idx * 17 + rank * 7919) & ((1 << 62) - 1)


_PRIO_STREAMS = {}


def _priority_stream(dev: torch.device) -> torch.cuda.Stream:
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _PRIO_STREAMS.get(key)
    if st is None:
        st = _PRIO_STREAMS[key] = torch.cuda.Stream(device=dev, priority=-1)
    return st


class PretrainEngine:
    def __init__(self, opt, device: Optional[torch.device] = None):
        self.opt = opt
        rank, local_rank, world, dev = comm.init_distributed(opt.dist_backend, getattr(opt, "comm_timeout", 600.0), device=device)
        self.rank, self.world, self.device = rank, world, dev
        self.stream = None
        if dev.type == "cuda" and os.environ.get("SDX_STREAM_PRIO", "1") != "0":
            # the whole step on a high-priority stream: the critical path (forward, BN,
            # dgrad chain) is dispatched ahead of the default-priority wgrad side stream.
            # 12.52 -> 12.43 ms/step same box, 4 alternating rounds (profiles/knob_sweep_r3.txt).
            # One stream per device and process, shared by every engine built in it.
            self.stream = _priority_stream(dev)
            torch.cuda.set_stream(self.stream)
        if opt.ngpu != world and world > 1:
            logging.warning(f"--ngpu {opt.ngpu} != launcher WORLD_SIZE {world}; using {world}")
        opt.world_size = world
        opt.local_batch = opt.batch_size // world
        setup_logging(opt.save_folder, rank)
        if rank == 0:
            logging.info(f"create {opt.conf_work_path} ...")
        torch.manual_seed(opt.seed)
        self.backend = resolve_backend(opt.backend, dev, opt.stem)

        model = SupConResNet(opt.model, opt.head, opt.feat_dim, opt.stem)
        if opt.ckpt:
            sd = ckpt_mod.load_checkpoint(opt.ckpt)["model"]
            ckpt_mod.load_model_state(model, sd)
            logging.info(f"load model from {opt.ckpt} ...")
        self.sync_group = None
        if opt.syncBN and world > 1:
            if self.backend == "torch":
                from ..parallel.syncbn import convert_sync_bn
                model = convert_sync_bn(model)
                self.syncbn_transport = "torch-syncbn"
            else:
                self.sync_group = dist.group.WORLD
                self._setup_syncbn_comm(opt, dev)
                if self.syncbn_transport == "none":
                    self.syncbn_transport = "process-group"
        if world > 1 and self.backend == "native":
            self._setup_gather_comm(opt, dev)
        emu = int(os.environ.get("SDX_SYNCBN_EMU", "0") or 0)
        if emu > 1 and world == 1 and self.backend == "native" and dev.type == "cuda":
            # SyncBN over `emu` identical virtual ranks on this GPU (comm.EmulatedGroup):
            # SDX_SYNCBN_EMU_KIND=fused (default, the xGMI fused exchange) | emu (reduce ->
            # x·W -> finalize, the kernel sequence of the RCCL path minus the collective)
            self.sync_group = comm.EmulatedGroup(emu)
            m = _ext.require()
            kind = os.environ.get("SDX_SYNCBN_EMU_KIND", "fused")
            h = m.xgmi_emu_small_comm(emu) if kind == "fused" else m.emu_small_comm(emu)
            comm.set_native_small_comm(self.sync_group, h)
            self.syncbn_transport = f"emulated-{emu}-{kind}"
            logging.info(f"SyncBN emulated over {emu} virtual ranks ({kind})")
        model = model.to(dev)
        if dev.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        self.model = model
        self.flat = FlatParams(model)
        self.optimizer = build_optimizer(opt.optimizer, self.flat, opt.learning_rate, opt.momentum,
                                         opt.weight_decay, backend="torch" if self.backend == "torch" else "auto")
        # SDX_EARLY_STEP=1 (native SGD): each bucket's update runs as soon as its gradients are
        # final (after its collective with several ranks), overlapping the rest of backward.
        # Off by default: on one MI355X the step's tail shrinks by ~85 us but the update
        # kernels slow the concurrent critical-path backward kernels more (12.31 -> 12.44-12.60
        # ms/step same box, profiles/early_step_r3.txt)
        early = None
        if (isinstance(self.optimizer, FusedSGD) and self.optimizer.native and not getattr(opt, "cuda_graph", False)
                and os.environ.get("SDX_EARLY_STEP", "0") == "1"):
            early = self.optimizer.apply_range
        self.reducer = (GradBucketReducer(self.flat, early_step=early, compress=getattr(opt, "grad_compress", "none"))
                        if (world > 1 or early is not None) else None)
        self.optimizer.grad_scale = (1.0 / world) if opt.grad_semantics == "ref" else 1.0
        self.runner = ModelRunner(model, self.backend, opt.precision, self.sync_group, master=self.flat.flat)
        self.criterion = DistributedContrastiveLoss(opt.method, opt.temp, opt.base_temperature, opt.contrast_mode,
                                                    backend="native" if self.backend == "native" else "torch")
        # data: whole uint8 dataset resident on the device
        ds = build_dataset(opt.dataset, opt.data_folder, True, opt.synthetic, opt.synthetic_size, opt.size, opt.seed,
                           native=True, workers=opt.num_workers)
        self.data = torch.from_numpy(ds.images).to(dev)
        # ImageFolder: native-resolution ragged store (RandomResizedCrop on original pixels)
        self.data_offs = torch.from_numpy(ds.offsets).to(dev) if ds.ragged else None
        self.data_hw = torch.from_numpy(ds.sizes).to(dev) if ds.ragged else None
        self.labels = torch.from_numpy(ds.labels).to(dev)
        self.sampler = DistributedIndexSampler(len(ds), opt.local_batch, world, rank, seed=opt.seed)
        self.aug = AugConfig.simclr(opt.size, opt.mean_t, opt.std_t)
        self.logger = None
        if rank == 0:
            from ..utils.tb import Logger
            self.logger = Logger(opt.tb_folder, flush_secs=2)
        self.start_epoch = 1
        self.global_step = 0
        # device-resident step state (so the step body is graph-capturable)
        self.record_norm_mean = torch.zeros((), device=dev)
        self._rnm_valid = torch.zeros((), device=dev)
        self._seed_t = torch.zeros((1,), dtype=torch.int64, device=dev)
        self._seed_host = 0
        self._seed_dev = False     # True once a hipGraph of the step exists (the seed then lives in _seed_t)
        self._ramp_t = torch.zeros((), device=dev)
        self._graph = None
        self._graph_stats = None
        self.prof = PhaseTimer(getattr(opt, "profile", False), dev)
        if getattr(opt, "resume", ""):
            self._resume(opt.resume)

    # ------------------------------------------------------------------------------
    # SyncBN statistics transport actually in use (bench.py reports it): none (W=1),
    # xgmi-fused, rccl-native, process-group (c10d collectives), emulated-W
    syncbn_transport = "none"

    def _setup_syncbn_comm(self, opt, dev):
        """SyncBN statistics transport for the native backend (SURVEY §2.3 X4/X6, §5.8;
        reference: main_supcon.py:222-224 converts the model to SyncBatchNorm).

        Candidates, each registered as a native handle so the C++ block executor exchanges
        each BN's sums itself on the compute stream:

        * ``xgmi-fused``: the one-shot IPC arena whose FUSED path reduces, exchanges and
          finalizes a BN's statistics in ONE launch (parallel/xgmi.py); all ranks must be
          peers on one node.
        * ``rccl-native``: a dedicated RCCL communicator (reduce -> ncclAllReduce ->
          finalize per BN).
        * ``process-group``: no native handle; the Python collective path (gloo runs).

        ``--syncbn_comm auto`` (default) sets up every candidate the job can have and MEASURES
        them on the first training batch (:meth:`autotune_syncbn`): all ranks agree on the
        fastest one (timings MAX-reduced over ranks, so the choice is identical everywhere).
        ``xgmi`` / ``rccl`` force one (RCCL is the fallback of both when the arena's self-check
        fails)."""
        want = getattr(opt, "syncbn_comm", "auto")
        self._syncbn_cands = {}
        if dev.type != "cuda":
            return
        timeout = float(getattr(opt, "comm_timeout", 600.0))
        if want in ("xgmi", "auto"):
            # set-up is agreed step by step across ranks (parallel/xgmi.py): either every
            # rank gets the arena or every rank raises here and falls back together
            try:
                from ..parallel.xgmi import OneShotAllReduce
                impl = OneShotAllReduce(timeout_s=timeout)
                self._xgmi = impl
                self._syncbn_cands["xgmi-fused"] = (impl.handle, impl)
            except Exception as e:  # noqa: BLE001
                (logging.warning if want == "xgmi" else logging.info)(
                    f"one-shot xGMI exchange unavailable ({e}); using RCCL")
        if (want == "auto" or not self._syncbn_cands) and comm.backend() == "nccl" \
                and os.environ.get("SDX_NATIVE_SYNCBN", "1") != "0":
            # 0 on every rank together when the dedicated communicator cannot be set up
            handle = comm.create_rccl_small_comm(None, timeout)
            if handle:
                self._syncbn_cands["rccl-native"] = (handle, None)
        if want == "auto" and comm.backend() != "nccl":
            self._syncbn_cands["process-group"] = (0, None)
        if not self._syncbn_cands:
            logging.warning("SyncBN statistics use the process-group all-reduce")
            return
        # until the measurement: RCCL when present (the conservative transport), else the first
        first = "rccl-native" if "rccl-native" in self._syncbn_cands else next(iter(self._syncbn_cands))
        self._activate_syncbn(first)
        self._syncbn_pending = want == "auto" and len(self._syncbn_cands) > 1
        logging.info(f"SyncBN statistics: {first} (candidates {list(self._syncbn_cands)})")

    _syncbn_cands: dict = {}
    _syncbn_pending = False
    syncbn_tune: Optional[dict] = None

    def _activate_syncbn(self, name: str):
        handle, impl = self._syncbn_cands[name]
        comm.set_small_allreduce(None, impl)
        comm.set_native_small_comm(None, handle)
        self.syncbn_transport = name

    def autotune_syncbn(self, idx: torch.Tensor, steps: int = 3, baseline: bool = False) -> Optional[dict]:
        """Pick the SyncBN transport by timing real training steps on batch ``idx`` with each
        candidate (one untimed step each first). The training state the steps touch
        (parameters, optimizer and BN buffers, the norm EMA) is restored afterwards, so the
        run follows the trajectory it would have had. Every rank measures its own step
        time; the times are MAX-reduced over the ranks (the step is as slow as its slowest
        rank) and every rank takes the argmin of the SAME reduced vector, so the choice is
        identical everywhere. ``baseline``: also time the step with rank-local BN statistics
        (no exchange, timing only) to report each transport's cost per exchanged BN.
        SDX_SYNCBN_TUNE_SKEW="rank:name:ms[,...]" adds ms to a rank's measurement (tests)."""
        self._syncbn_pending = False
        names = list(self._syncbn_cands)
        if self.device.type != "cuda" or (len(names) < 2 and not baseline) or not names:
            return None
        if baseline:
            names = names + ["local-bn"]
        state = [self.flat.flat, self.optimizer.buf, self.record_norm_mean, self._rnm_valid]
        state += [t for t in self.model.buffers()]
        if getattr(self.optimizer, "norms", None) is not None:
            state.append(self.optimizer.norms)
        snap = [t.detach().clone() for t in state]
        pend = self.runner._nbt_pending
        active = self.syncbn_transport
        group = self.runner.sync_group
        self._host_prelude(1, 0, 1)
        # two interleaved passes over the candidates, the faster of each candidate's two
        # timings kept: a drifting clock or a cold first candidate does not pick the transport
        ms = [float("inf")] * len(names)
        for _ in range(2):
            for k, nm in enumerate(names):
                if nm == "local-bn":
                    self.runner.sync_group = None
                else:
                    self._activate_syncbn(nm)
                self._step_body(idx)
                torch.cuda.synchronize()
                comm.barrier()
                t0 = time.perf_counter()
                for _ in range(steps):
                    self._step_body(idx)
                torch.cuda.synchronize()
                comm.barrier()
                ms[k] = min(ms[k], (time.perf_counter() - t0) / steps * 1e3)
                self.runner.sync_group = group
        with torch.no_grad():
            for t, v in zip(state, snap):
                t.copy_(v)
        self.runner._nbt_pending = pend
        for item in filter(None, os.environ.get("SDX_SYNCBN_TUNE_SKEW", "").split(",")):
            r, nm, extra = item.split(":")
            if int(r) == self.rank and nm in names:
                ms[names.index(nm)] += float(extra)
        real = [i for i, nm in enumerate(names) if nm != "local-bn"]
        best, red = comm.agree_fastest(names, ms, eligible=real)
        self._activate_syncbn(best if best in self._syncbn_cands else active)
        n_bn = 2 * sum(1 for mod in self.model.encoder.modules() if isinstance(mod, torch.nn.BatchNorm2d))
        self.syncbn_tune = {"chosen": best, "step_ms": {nm: round(v, 3) for nm, v in zip(names, red)},
                            "exchanges_per_step": n_bn}
        if baseline:
            # (transport − local-BN step) per exchanged BN; within timing noise it can be ≤ 0
            base = red[names.index("local-bn")]
            self.syncbn_tune["us_per_bn"] = {names[i]: round((red[i] - base) * 1e3 / n_bn, 2) for i in real}
        logging.info(f"SyncBN transport measured: {self.syncbn_tune}")
        return self.syncbn_tune

    def _setup_gather_comm(self, opt, dev):
        """Native transport of the contrastive loss's embedding all-gather / reduce-scatter
        (SURVEY §2.3 X5): the dedicated RCCL communicator (the SyncBN one when it is RCCL,
        else a new one; created and self-checked by all ranks together, 0 everywhere on
        failure -> c10d). gloo process groups keep the c10d path."""
        if dev.type != "cuda" or comm.backend() != "nccl" or os.environ.get("SDX_NATIVE_GATHER", "1") == "0":
            return
        m = _ext.require()
        h = comm.native_small_comm(None)
        if not (h and m.small_comm_kind(h) == 1):
            h = comm.create_rccl_small_comm(None, float(getattr(opt, "comm_timeout", 600.0)))
        if h:
            comm.set_native_gather_comm(None, h)
            logging.info("contrastive-loss embedding gather: dedicated RCCL communicator (native)")

    def _resume(self, path):
        st = ckpt_mod.load_checkpoint(path)
        ckpt_mod.load_model_state(self.model, st["model"])
        self.optimizer.load_state_dict(st["optimizer"])
        self.start_epoch = int(st["epoch"]) + 1
        extra = st.get("sdx_state") or {}
        self.global_step = int(extra.get("global_step", 0))
        rnm = extra.get("record_norm_mean")
        if rnm is not None:
            self.record_norm_mean.fill_(float(rnm))
            self._rnm_valid.fill_(1.0)
        logging.info(f"resumed from {path} at epoch {self.start_epoch}")

    def _extra_state(self, epoch):
        valid = float(self._rnm_valid) > 0
        return {"global_step": self.global_step, "epoch": epoch,
                "record_norm_mean": float(self.record_norm_mean) if valid else None}

    # ------------------------------------------------------------------------------
    def make_views(self, idx: torch.Tensor, epoch: int = 1, it: int = 0) -> torch.Tensor:
        if not getattr(self.opt, "gpu_aug", 1):
            return self._make_views_cpu(idx, epoch, it)
        if self.backend == "native":
            # the seed is read from device memory by the kernel (graph-replay safe)
            # eager: the seed is a kernel argument; a captured step reads it from _seed_t at replay
            x = augment_gpu(self.data, idx, self.aug, self._seed_host, self._seed_t if self._seed_dev else None,
                            self.data_offs, self.data_hw)
        else:
            x = augment(self.data, idx, self.aug, step_seed(self.opt.seed, epoch, it, self.rank), self.data_offs,
                        self.data_hw)
            x = nhwc8_to_nchw(x)
        return x

    def _make_views_cpu(self, idx, epoch, it):
        """``--gpu_aug 0``: the torch CPU pipeline (same draws as the kernel) on a host copy
        of the dataset, ``--num_workers`` intra-op threads, then moved to the device."""
        if getattr(self, "_cpu_data", None) is None:
            torch.set_num_threads(max(1, int(self.opt.num_workers)))
            self._cpu_data = self.data.cpu()
            self._cpu_offs = self.data_offs.cpu() if self.data_offs is not None else None
            self._cpu_hw = self.data_hw.cpu() if self.data_hw is not None else None
        x = augment(self._cpu_data, idx.cpu(), self.aug, step_seed(self.opt.seed, epoch, it, self.rank),
                    self._cpu_offs, self._cpu_hw)
        if self.backend == "native":
            return x.to(self.device, torch.bfloat16)
        return nhwc8_to_nchw(x).to(self.device)

    def _host_prelude(self, epoch: int, it: int, iters: int):
        """Per-step host-side scalars, written to device tensors the step body reads."""
        opt = self.opt
        warmup_learning_rate(opt, epoch, it, iters, self.optimizer)
        self.optimizer._sync_lr()
        self._seed_host = step_seed(opt.seed, epoch, it, self.rank)
        if self._seed_dev:
            self._seed_t.fill_(self._seed_host)
        if opt.sec or opt.l2reg:
            now_iter = (epoch - 1) * iters + it
            self._ramp_t.fill_(now_iter / (opt.epochs * iters))

    def _step_body(self, idx: torch.Tensor, epoch: int = 1, it: int = 0):
        """Device work of one step: no host syncs, no host-dependent control flow
        (capturable into a hipGraph)."""
        opt = self.opt
        mb = getattr(opt, "micro_batch", 0) or 0
        if 0 < mb < 2 * idx.numel():
            return self._step_body_gradcache(idx, epoch, it, mb)
        ph = self.prof.phase
        with ph("augment"):
            prefetch = getattr(self.runner, "prefetch_weights", None)
            if prefetch is not None:
                prefetch()          # weight conversion overlaps the augmentation launch
            zeroed = self._zero_grad_side()
            x = self.make_views(idx, epoch, it)
            # (SimCLR ignores labels: no gather kernel in its step)
            labels = self.labels[idx] if opt.method == "SupCon" else None
        with ph("forward"):
            feats = self.runner.forward(x)
        with ph("loss"):
            loss = self.criterion(feats, labels if opt.method == "SupCon" else None)
            stats = self._norm_terms(feats)
            extra = stats.pop("extra_loss")
            if extra is not None:
                loss = loss + extra
        with ph("backward"):
            if zeroed is not None:
                torch.cuda.current_stream(self.device).wait_event(zeroed)
            else:
                self.optimizer.zero_grad()
            # a persistent seed gradient: no ones-fill kernel per step
            one = getattr(self, "_one_grad", None)
            if one is None or one.device != loss.device or one.dtype != loss.dtype:
                one = self._one_grad = torch.ones((), device=loss.device, dtype=loss.dtype)
            loss.backward(one)
        if self.reducer is not None:
            with ph("grad_sync_wait"):
                self.reducer.finish()
        with ph("optimizer"):
            self.optimizer.step()
        stats["loss_local"] = loss.detach()
        return stats

    def _zero_grad_side(self):
        """Zero the gradient buffer on the wgrad side stream at the start of the step (after
        the previous optimizer update), where it overlaps the forward instead of sitting on
        the compute stream before the backward (SDX_ZERO_SIDE=0: there). Returns the event
        the backward waits on, or None when it is left to the backward. The side stream's
        weight gradients are queued behind it anyway (FIFO)."""
        from ..ops import streams
        if not (_ZERO_SIDE and streams.ENABLED and self.device.type == "cuda"):
            return None
        main = torch.cuda.current_stream(self.device)
        s = streams.side(self.device)
        s.wait_stream(main)
        with torch.cuda.stream(s):
            self.optimizer.zero_grad()
        ev = getattr(self, "_zg_ev", None)
        if ev is None:
            ev = self._zg_ev = torch.cuda.Event()
        ev.record(s)
        return ev

    def _step_body_gradcache(self, idx: torch.Tensor, epoch: int, it: int, mb: int):
        """Gradient-cache step for contrastive batches larger than one encoder pass fits in
        HBM (e.g. BS 4096 at 224x224, BASELINE config 5): (1) encode all views in chunks of
        ``mb`` without autograd, (2) contrastive loss + norm terms on the full feature set,
        backward to the features only, (3) re-encode each chunk with autograd and backprop
        its slice of the feature gradient. Activation memory is one chunk's; the loss and
        its gradient are those of the full batch. BatchNorm statistics are per chunk (as
        in any micro-batched BN network); running statistics are updated once per chunk
        in the re-encode pass only. The update is therefore the EXACT gradient of the
        full-batch loss of the same network with ghost batch norm of ``mb`` views — not the
        reference's full-batch BN (tests/test_gradcache.py pins this equivalence); for
        full-batch BN semantics run the whole local batch in one pass (288 GB of HBM holds
        the config-5 batch: profiles/cfg5_slice_r2.json). The bucket reducer stays paused
        until the last chunk.
        """
        opt = self.opt
        ph = self.prof.phase
        with ph("augment"):
            x = self.make_views(idx, epoch, it)
            labels = self.labels[idx]
        chunks = list(torch.split(x, mb))
        bns = [m for m in self.model.modules() if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)]
        saved = [(m.running_mean.clone(), m.running_var.clone(), m.num_batches_tracked.clone())
                 for m in bns if m.running_mean is not None]
        pend = self.runner._nbt_pending
        with ph("forward"), torch.no_grad():
            feats = torch.cat([self.runner.forward(c) for c in chunks])
        with torch.no_grad():          # undo the statistics updates of the no-grad pass
            for m, (rm, rv, nb) in zip([m for m in bns if m.running_mean is not None], saved):
                m.running_mean.copy_(rm)
                m.running_var.copy_(rv)
                m.num_batches_tracked.copy_(nb)
        self.runner._nbt_pending = pend
        feats = feats.detach().requires_grad_(True)
        with ph("loss"):
            loss = self.criterion(feats, labels if opt.method == "SupCon" else None)
            stats = self._norm_terms(feats)
            extra = stats.pop("extra_loss")
            if extra is not None:
                loss = loss + extra
            loss.backward()
        gfeat = feats.grad
        self.optimizer.zero_grad()
        with ph("backward"):
            off = 0
            for i, c in enumerate(chunks):
                n = c.shape[0]
                last = i == len(chunks) - 1
                ctx = self.reducer.no_sync() if (self.reducer is not None and not last) else _null()
                with ctx:
                    f = self.runner.forward(c)
                    f.backward(gfeat[off:off + n].to(f.dtype))
                off += n
        if self.reducer is not None:
            with ph("grad_sync_wait"):
                self.reducer.finish()
        with ph("optimizer"):
            self.optimizer.step()
        stats["loss_local"] = loss.detach()
        return stats

    def train_step(self, idx: torch.Tensor, epoch: int, it: int, iters: int):
        maybe_inject(self.rank, self.global_step)
        self._host_prelude(epoch, it, iters)
        if self._graph is not None:
            self._idx_buf.copy_(idx, non_blocking=True)
            self._graph.replay()
            self.runner._nbt_pending += self._graph_nbt
            st = self._graph_stats
        else:
            st = self._step_body(idx, epoch, it)
        self.global_step += 1
        return st

    def enable_cuda_graph(self, idx_example: torch.Tensor, warmup: int = 2) -> bool:
        """Capture the whole training step (aug → fwd → loss → bwd → SGD) in one hipGraph.

        Single-process only (the data-parallel path keeps eager launches; an emulated SyncBN
        group — SDX_SYNCBN_EMU — is captured too: the fused exchange takes its epoch from
        device-side counters, so every replay advances it, bn.hip xg_exchange). Capture needs
        warm-up steps run on a side stream; they execute real updates, so the training
        state they touch (parameters, optimizer buffers, BN running statistics, the norm
        EMA) is snapshotted first and restored after the capture — a graphed run follows
        exactly the eager trajectory."""
        if self.device.type != "cuda" or self.world > 1 or self.backend != "native":
            return False
        self._idx_buf = idx_example.clone()
        self._seed_dev = True
        state = [self.flat.flat, self.optimizer.buf, self.record_norm_mean, self._rnm_valid]
        state += [t for t in self.model.buffers()]
        if getattr(self.optimizer, "norms", None) is not None:
            state.append(self.optimizer.norms)
        snap = [t.detach().clone() for t in state]
        pend = self.runner._nbt_pending
        self._host_prelude(1, 0, 1)
        # The step is captured as ONE chain: the weight gradients run in line on the capture
        # stream instead of forking to the wgrad side stream (SDX_GRAPH_SIDE=1 keeps the
        # fork). A captured two-stream DAG replays its branches on several hardware queues
        # with a cross-queue wait at every fork: 24.9 vs 11.9 ms eager at 256 images/GPU
        # (23.5 ms even with per-node priorities), while each kernel replayed on its own runs
        # at its eager speed (profiles/graph_probe_r6.txt, profiles/graph_ab_r6.txt).
        # In line, the dedicated wgrad kernels get the whole chip (their eager block target
        # keeps half of it for the concurrent critical path): SDX_GRAPH_WGRAD_BLOCKS, 256.
        from ..ops import streams
        side_prev = streams.ENABLED
        streams.ENABLED = os.environ.get("SDX_GRAPH_SIDE", "0") == "1"
        m = _ext.require()
        tgt_prev = m.wgrad_block_target_set(int(os.environ.get("SDX_GRAPH_WGRAD_BLOCKS", "256"))) \
            if not streams.ENABLED else None
        try:
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    self._step_body(self._idx_buf)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            p0 = self.runner._nbt_pending
            # thread-local capture: the communicator watchdog thread (csrc/bindings/comm_ops.cpp)
            # keeps polling its events while this thread captures
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._graph_stats = self._step_body(self._idx_buf)
        finally:
            streams.ENABLED = side_prev
            if tgt_prev is not None:
                m.wgrad_block_target_set(tgt_prev)
        # BN passes of one step, counted on the host (ModelRunner.flush_bn_counters) per replay
        self._graph_nbt = self.runner._nbt_pending - p0
        self._graph = g
        with torch.no_grad():
            for t, v in zip(state, snap):
                t.copy_(v)
        self.runner._nbt_pending = pend
        return True

    def _norm_terms(self, feats):
        """SEC / L2-reg regularisers on un-normalised global features (main_supcon.py:295-317).
        The EMA ``record_norm_mean`` and the ramp live in device tensors."""
        opt = self.opt
        if not (opt.sec or opt.l2reg) and feats.is_cuda and feats.dim() == 2 and _ext.available():
            return self._norm_stats_native(feats)
        norms = feats.float().norm(dim=1)
        n_global = norms.numel() * self.world
        local = torch.stack([norms.sum(), (norms * norms).sum()])
        need_global = opt.sec or opt.l2reg
        if need_global and self.world > 1:
            g = local.detach().clone()
            comm.all_reduce_sum_(g)
        else:
            g = local.detach() * (self.world if self.world > 1 else 1)
        norm_mean = g[0] / n_global
        norm_var = g[1] / n_global - norm_mean * norm_mean
        m = opt.norm_momentum
        rec = self.record_norm_mean
        rec.copy_(torch.where(self._rnm_valid > 0, (1 - m) * rec + m * norm_mean, norm_mean))
        self._rnm_valid.fill_(1.0)
        extra = torch.zeros((), device=feats.device)
        loss_sec = ((norms - rec) ** 2).sum() / n_global
        loss_l2 = (norms ** 2).sum() / n_global
        if opt.sec:
            extra = extra + opt.sec_wei * self._ramp_t * loss_sec
        if opt.l2reg:
            extra = extra + opt.l2reg_wei * self._ramp_t * loss_l2
        return {"extra_loss": extra, "norm_mean": norm_mean.detach(), "norm_var": norm_var.detach(),
                "loss_sec": loss_sec.detach(), "loss_l2reg": loss_l2.detach(),
                "record_norm_mean": rec.detach().clone()}

    def _norm_stats_native(self, feats):
        """Logging-only norm statistics (no SEC / L2-reg term in the loss): one launch
        (csrc/kernels/featnorm.hip) computes them and advances the record_norm_mean EMA.
        Same semantics as the torch path: global sums are estimated as local·W (no
        collective) when no regulariser needs the exact global statistics."""
        from ..ops.streams import SideWork
        m = _ext.require()
        x = feats.detach().float().contiguous()
        n_global = float(x.shape[0] * self.world)
        mom = float(self.opt.norm_momentum)
        sums = getattr(self, "_ns_sums", None)
        if sums is None or sums.device != x.device:
            sums = self._ns_sums = torch.zeros(2, dtype=torch.float64, device=x.device)
        # nothing in the step reads these: on the wgrad side stream (idle here), off the loss
        # -> backward path; the end-of-backward join orders every later reader behind them
        with (SideWork(x) if _NORM_SIDE else contextlib.nullcontext()):
            if self.world > 1:
                m.norm_stats(x, 0, sums, n_global, mom, self.record_norm_mean, self._rnm_valid)
                sums.mul_(float(self.world))
                out = m.norm_stats(x, 2, sums, n_global, mom, self.record_norm_mean, self._rnm_valid)
            else:
                out = m.norm_stats(x, 1, sums, n_global, mom, self.record_norm_mean, self._rnm_valid)
        return {"extra_loss": None, "norm_mean": out[0], "norm_var": out[1], "loss_sec": out[3],
                "loss_l2reg": out[4], "record_norm_mean": out[2]}

    # ------------------------------------------------------------------------------
    def train_epoch(self, epoch: int) -> float:
        opt = self.opt
        self.model.train()
        self.sampler.set_epoch(epoch)
        iters = len(self.sampler)
        if opt.max_steps:
            iters = min(iters, opt.max_steps)
        batch_time, data_time, losses = AverageMeter(), AverageMeter(), AverageMeter()
        loss_acc = torch.zeros((), device=self.device)
        window_loss = torch.zeros((), device=self.device)
        window_n = 0
        end = time.time()
        t_window = time.time()
        for it, idx in enumerate(self.sampler.batches(self.device)):
            if it >= iters:
                break
            if self._syncbn_pending:
                # --syncbn_comm auto: measure the transports on this batch (state restored)
                self.autotune_syncbn(idx)
            data_time.update(time.time() - end)
            if opt.cuda_graph and self._graph is None and not getattr(self, "_graph_failed", False):
                try:
                    ok = self.enable_cuda_graph(idx)
                    logging.info("hipGraph capture of the train step: " + ("enabled" if ok else "not applicable"))
                except Exception as e:  # noqa: BLE001
                    self._graph_failed = True
                    logging.warning(f"hipGraph capture failed, running eagerly: {e!r}")
            st = self.train_step(idx, epoch, it, iters)
            loss_acc += st["loss_local"]
            window_loss += st["loss_local"]
            window_n += 1
            batch_time.update(time.time() - end)
            end = time.time()
            if (it + 1) % opt.print_freq == 0 or it + 1 == iters:
                vals = torch.stack([window_loss, st["norm_mean"], st["record_norm_mean"], st["norm_var"],
                                    st["loss_sec"], st["loss_l2reg"], st["loss_local"]])
                vals[0] = vals[0] / max(window_n, 1)
                if self.world > 1:
                    red = vals[[0, 6]].clone()
                    comm.all_reduce_sum_(red)
                    vals[0], vals[6] = red[0], red[1]
                v = vals.tolist()    # one host sync per print window
                if self.device.type == "cuda":
                    torch.cuda.synchronize()
                dt = (time.time() - t_window) / window_n
                t_window = time.time()
                losses.update(v[0], window_n)
                losses.val = v[6]
                batch_time.val = dt
                if self.rank == 0:
                    now_iter = (epoch - 1) * iters + it
                    for tag, k in (("info/norm_mean", 1), ("info/norm_var", 3), ("info/record_norm_mean", 2),
                                   ("info/loss_sec", 4), ("info/loss_l2reg", 5)):
                        self.logger.log_value(tag, v[k], now_iter)
                    logging.info(
                        "Train: [{0}][{1}/{2}]\tBT {bt:.3f} ({bta:.3f})\tDT {dtv:.3f} ({dta:.3f})\t"
                        "loss {lv:.3f} ({la:.3f})\tnorm_mean {nm:.3f} (record: {rec:.3f}) var {var:.3f}\t"
                        "img/s {ips:.0f}".format(
                            epoch, it + 1, iters, bt=dt, bta=batch_time.avg, dtv=data_time.val, dta=data_time.avg,
                            lv=v[6], la=losses.avg, nm=v[1], rec=v[2], var=v[3],
                            ips=opt.batch_size / max(dt, 1e-9)))
                    if self.prof.enabled:
                        logging.info("phases (ms/step): " + PhaseTimer.format(self.prof.summary()))
                    sys.stdout.flush()
                window_loss = torch.zeros((), device=self.device)
                window_n = 0
        # BN num_batches_tracked is host-counted on the native path: visible in the buffers
        # from every epoch end on, not only through state_dict()
        flush = getattr(self.runner, "flush_bn_counters", None)
        if flush is not None:
            flush()
        return losses.avg

    def run(self):
        opt = self.opt
        for epoch in range(self.start_epoch, opt.epochs + 1):
            adjust_learning_rate(opt, self.optimizer, epoch)
            t1 = time.time()
            loss = self.train_epoch(epoch)
            t2 = time.time()
            logging.info("epoch {}, total time {:.2f}".format(epoch, t2 - t1))
            if self.rank == 0:
                self.logger.log_value("loss", loss, epoch)
                self.logger.log_value("learning_rate", self.optimizer.param_groups[0]["lr"], epoch)
            if epoch % opt.save_freq == 0 and self.rank == 0:
                f = os.path.join(opt.save_folder, f"ckpt_epoch_{epoch}.pth")
                ckpt_mod.save_model(self.model, self.optimizer, opt, epoch, f, self._extra_state(epoch))
            comm.barrier()
        if self.rank == 0:
            f = os.path.join(opt.save_folder, "last.pth")
            ckpt_mod.save_model(self.model, self.optimizer, opt, opt.epochs, f, self._extra_state(opt.epochs))
            self.logger.close()
        comm.barrier()
        return os.path.join(opt.save_folder, "last.pth")
