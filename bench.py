#!/usr/bin/env python3
"""Headline benchmark: SimCLR ResNet-50 (CIFAR stem) pretraining throughput on MI355X.

Measures the full training step of the reference's headline config (BASELINE.json:
ResNet-50, batch 256 per GPU, 2 views of 32x32, τ=0.5, SyncBN + data parallel for N>1):
GPU augmentation of both views → native gfx950 forward → distributed NT-Xent loss →
backward with overlapped RCCL gradient all-reduce → fused SGD step. Data are synthetic
CIFAR-shaped uint8 images (no network for datasets); weights are random-init.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 launched
with torch.distributed.run, one rank per GPU. W untimed steps, then exactly K steps
bracketed by barrier + synchronize; the time is the MAX over ranks; rank 0 prints one
JSON line. ``value`` = whole-job source images/sec (each image is processed as 2 views).

Other BASELINE.json configs (same step, same JSON line):

* ``--global_batch 256`` on 2 GPUs: the README headline config (BS 256 over 2 ranks,
  128 per GPU, strong scaling); ``--per_gpu_batch 128`` is its 1-GPU slice.
* ``--dataset cifar100 --global_batch 1024``: config 4 (8 GPUs, 128 per GPU).
* ``--config supcon224``: config 5 — SupCon, ImageNet stem at 224x224, LARS, 512 images
  (1024 views) per GPU: the whole local batch in ONE encoder pass (full-batch BN
  semantics, as the reference recipe) — it needs ≈51 GB of the 288 GB of HBM, measured
  (profiles/cfg5_slice_r2.json). ``--micro_batch V`` switches to gradient-cache chunks
  of V views (per-chunk BN statistics, see engine/pretrain.py) for larger batches.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) SimCLR ResNet-50 BS=256; CIFAR-10 linear-probe top-1"


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _self_launch(n: int) -> int:
    """``--gpus N`` (N > 1) without a launcher: start one rank per GPU through
    torch.distributed.run as a CHILD process (never an exec: nothing here has touched the
    GPU, and the parent stays alive to relay), pass rank 0's JSON line through, and return
    the child's exit status. Reference launch recipe: run_supcon.sh:4-11."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    env = dict(os.environ, SDX_BENCH_CHILD="1")
    return subprocess.call(cmd, env=env)


def main():
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    n_req = pre.parse_known_args()[0].gpus
    if n_req > 1 and "WORLD_SIZE" not in os.environ and not os.environ.get("SDX_BENCH_CHILD"):
        raise SystemExit(_self_launch(n_req))

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--per_gpu_batch", type=int, default=None,
                    help="images per GPU (weak scaling; default 256, 512 for --config supcon224)")
    ap.add_argument("--global_batch", type=int, default=None,
                    help="fixed total images per step split over the ranks (strong scaling)")
    ap.add_argument("--dataset", default="cifar10", choices=["cifar10", "cifar100"])
    ap.add_argument("--config", default="simclr32", choices=["simclr32", "supcon224"])
    ap.add_argument("--micro_batch", type=int, default=0,
                    help="views per encoder chunk (gradient cache); 0 = the whole local batch in one pass")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--backend", default="native", choices=["native", "torch"])
    ap.add_argument("--no_syncbn", action="store_true")
    ap.add_argument("--graph", type=int, default=0,
                    help="capture the step in a hipGraph (single GPU; measured slower than eager + wgrad side stream)")
    a, extra = ap.parse_known_args()

    import torch
    import torch.distributed as dist

    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    from simclr_pytorch_distributed_amd.parallel import comm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    n = world
    big = a.config == "supcon224"
    if a.global_batch is not None:
        if a.global_batch % n:
            raise SystemExit(f"--global_batch {a.global_batch} is not divisible by {n} ranks")
        per_gpu, scaling = a.global_batch // n, "strong"
    else:
        per_gpu, scaling = (a.per_gpu_batch or (512 if big else 256)), "weak"
    global_batch = per_gpu * n
    work = os.path.join(tempfile.gettempdir(), f"sdx_bench_{os.getpid()}")
    size = 224 if big else 32
    argv = ["--batch_size", str(global_batch), "--model", a.model, "--temp", "0.5" if not big else "0.1",
            "--learning_rate", "0.5", "--cosine", "--method", "SupCon" if big else "SimCLR", "--epochs", "100",
            "--synthetic", "--synthetic_size", str(max(2 * global_batch if big else 8192, 4 * per_gpu)),
            "--backend", a.backend, "--dataset", a.dataset,
            "--work_dir", work, "--print_freq", "1000000", "--ngpu", str(n)]
    if big:
        argv += ["--stem", "imagenet", "--size", "224", "--optimizer", "lars"]
    mb = a.micro_batch
    if mb:
        argv += ["--micro_batch", str(mb)]
    if n > 1 and not a.no_syncbn:
        argv.append("--syncBN")
    opt = parse_pretrain(argv + extra, make_dirs=False)
    import logging
    logging.disable(logging.INFO)
    eng = PretrainEngine(opt)
    dev = eng.device
    eng.model.train()
    eng.sampler.set_epoch(1)
    batches = eng.sampler.batches(dev)
    iters = len(eng.sampler)

    def next_idx(i):
        nonlocal batches
        try:
            return next(batches)
        except StopIteration:
            batches = eng.sampler.batches(dev)
            return next(batches)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()

    # N > 1: the SyncBN transport candidates of --syncbn_comm (default rccl: RCCL only; auto: the
    # fused xGMI exchange too) are timed on real steps (state restored afterwards), the ranks
    # agree on the fastest; reported in the JSON line with a local-BN baseline
    tune = eng.autotune_syncbn(next_idx(0), steps=3, baseline=True) if n > 1 and not a.no_syncbn else None
    graphed = False
    if a.graph:
        # capture the whole step in one hipGraph (its 2 capture warm-up steps are real steps)
        try:
            graphed = eng.enable_cuda_graph(next_idx(0))
        except Exception as e:  # noqa: BLE001
            print(f"warning: hipGraph capture failed, eager fallback: {e!r}", file=sys.stderr)
    first_loss = None
    for i in range(a.warmup):
        st0 = eng.train_step(next_idx(i), 1, i % iters, iters)
        if first_loss is None:
            # a snapshot (read after the timed region, no sync here): under --graph the stats
            # dict is the captured graph's persistent output, overwritten by every replay
            first_loss = st0["loss_local"].detach().clone()
    sync()
    # host cost of issuing one step into an idle queue (diagnostic, stderr)
    th = []
    for i in range(3):
        sync()
        t = time.perf_counter()
        eng.train_step(next_idx(i), 1, i % iters, iters)
        th.append(time.perf_counter() - t)
        sync()
    print(f"host issue time (idle queue) {min(th) * 1e3:.3f} ms/step", file=sys.stderr)
    t0 = time.perf_counter()
    for i in range(a.steps):
        st = eng.train_step(next_idx(i), 1, i % iters, iters)
    t_host = time.perf_counter() - t0      # host issue time (no sync inside the loop)
    sync()
    dt = time.perf_counter() - t0
    print(f"host issue time {t_host / a.steps * 1e3:.3f} ms/step", file=sys.stderr)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if n > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    loss = float(st["loss_local"].item())
    loss0 = float(first_loss.item()) if first_loss is not None else None
    ms = dt / a.steps * 1e3
    value = global_batch * a.steps / dt
    d_in = {"resnet18": 512, "resnet34": 512}.get(a.model, 2048)
    peak_gb = torch.cuda.max_memory_allocated(dev) / 1e9 if dev.type == "cuda" else 0.0
    if big:
        desc = f"{a.model} (ImageNet stem, 224x224) + MLP head {d_in}-{d_in}-128, SupCon tau=0.1, LARS"
        metric = METRIC.replace("SimCLR ResNet-50 BS=256", "SupCon ResNet-50 224x224")
    else:
        desc = f"{a.model} (CIFAR stem) + MLP head {d_in}-{d_in}-128, SimCLR tau=0.5"
        metric = METRIC
    if comm.rank() == 0:
        print(json.dumps({
            "metric": metric, "value": round(value, 2), "unit": "images/sec", "n_gpus": n, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"model": desc, "dataset_shape": a.dataset,
                       "global_batch": global_batch, "per_gpu_batch": per_gpu, "views": 2,
                       "image_size": size, "seq_len": None, "micro_batch_views": mb or None,
                       "parallelism": f"dp{n}" + ("+syncbn" if n > 1 and not a.no_syncbn else ""),
                       "backend": eng.backend, "syncbn_transport": eng.syncbn_transport,
                       "syncbn_step_ms": tune["step_ms"] if tune else None,
                       "syncbn_us_per_bn": tune.get("us_per_bn") if tune else None, "hip_graph": graphed,
                       "views_per_sec": round(2 * value, 2),
                       "peak_hbm_gb": round(peak_gb, 2), "hbm_capacity_gb": 288,
                       # first warm-up step and last timed step: the run trains from random init
                       # (44.5455 = every embedding identical, the collapse the reference recipe
                       # lr 0.5 / no warm-up also reaches in fp32 torch on synthetic data in the
                       # first ~20-60 steps: profiles/convergence_r1.txt)
                       "first_loss_local": round(loss0, 4) if loss0 is not None else None,
                       "last_loss_local": round(loss, 4), "loss_steps": a.warmup + 3 + a.steps},
        }), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
