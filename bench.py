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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--per_gpu_batch", type=int, default=256)
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
    global_batch = a.per_gpu_batch * n
    work = os.path.join(tempfile.gettempdir(), f"sdx_bench_{os.getpid()}")
    argv = ["--batch_size", str(global_batch), "--model", a.model, "--temp", "0.5", "--learning_rate", "0.5",
            "--cosine", "--method", "SimCLR", "--epochs", "100", "--synthetic",
            "--synthetic_size", str(max(8192, 4 * global_batch)), "--backend", a.backend,
            "--work_dir", work, "--print_freq", "1000000", "--ngpu", str(n)]
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

    graphed = False
    if a.graph:
        # capture the whole step in one hipGraph (its 2 capture warm-up steps are real steps)
        try:
            graphed = eng.enable_cuda_graph(next_idx(0))
        except Exception as e:  # noqa: BLE001
            print(f"warning: hipGraph capture failed, eager fallback: {e!r}", file=sys.stderr)
    for i in range(a.warmup):
        eng.train_step(next_idx(i), 1, i % iters, iters)
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
    ms = dt / a.steps * 1e3
    value = global_batch * a.steps / dt
    d_in = {"resnet18": 512, "resnet34": 512}.get(a.model, 2048)
    if comm.rank() == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(value, 2), "unit": "images/sec", "n_gpus": n, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
            "config": {"model": f"{a.model} (CIFAR stem) + MLP head {d_in}-{d_in}-128, SimCLR tau=0.5",
                       "global_batch": global_batch, "per_gpu_batch": a.per_gpu_batch, "views": 2,
                       "image_size": 32, "seq_len": None,
                       "parallelism": f"dp{n}" + ("+syncbn" if n > 1 and not a.no_syncbn else ""),
                       "backend": eng.backend, "hip_graph": graphed, "views_per_sec": round(2 * value, 2),
                       "last_loss_local": round(loss, 4)},
        }), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
