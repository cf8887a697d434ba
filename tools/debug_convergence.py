#!/usr/bin/env python3
"""Isolate which component of the native path changes SimCLR training dynamics.

Runs K steps from the same seed with the native engine and with one component swapped
for its torch counterpart (loss, optimizer, model forward/backward, fused-block path,
augmentation) and prints the loss trajectory of each variant.
"""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def run(variant, steps, every, seed=0):
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.data.augment import augment, nhwc8_to_nchw
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine, step_seed
    from simclr_pytorch_distributed_amd.losses.supcon import DistributedContrastiveLoss
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.optim.flat import build_optimizer
    import logging
    logging.disable(logging.INFO)
    backend = "torch" if variant == "torch" else "native"
    argv = ["--batch_size", "256", "--learning_rate", "0.5", "--temp", "0.5", "--cosine", "--method", "SimCLR",
            "--synthetic", "--synthetic_size", "10240", "--epochs", "12", "--seed", str(seed), "--backend", backend,
            "--work_dir", tempfile.mkdtemp(), "--print_freq", "1000000"]
    if variant == "fp32_torch":
        argv[argv.index("--backend") + 1] = "torch"
        argv += ["--precision", "fp32"]
    opt = parse_pretrain(argv, make_dirs=False)
    eng = PretrainEngine(opt)
    o = eng.opt
    if variant == "loss_torch":
        eng.criterion = DistributedContrastiveLoss(o.method, o.temp, o.base_temperature, o.contrast_mode,
                                                   backend="torch")
    elif variant == "optim_torch":
        eng.optimizer = build_optimizer(o.optimizer, eng.flat, o.learning_rate, o.momentum, o.weight_decay,
                                        backend="torch")
    elif variant == "unfused":
        eng.runner = ModelRunner(eng.model, "native", o.precision, None, master=eng.flat.flat, fused=False)
    elif variant == "model_torch":
        eng.runner = ModelRunner(eng.model, "torch", o.precision, None, master=eng.flat.flat)
        mv = eng.make_views
        eng.make_views = lambda idx, e=1, it=0: nhwc8_to_nchw(mv(idx, e, it))
    elif variant == "aug_torch":
        eng.make_views = lambda idx, e=1, it=0: augment(eng.data, idx, eng.aug, step_seed(seed, e, it, 0))
    eng.model.train()
    iters = len(eng.sampler)
    out = []
    n = 0
    for epoch in range(1, 100):
        eng.sampler.set_epoch(epoch)
        for it, idx in enumerate(eng.sampler.batches(eng.device)):
            st = eng.train_step(idx, epoch, it, iters)
            if n % every == 0 or n == steps - 1:
                out.append((n, round(float(st["loss_local"]), 3), round(float(st["norm_mean"]), 1)))
            n += 1
            if n >= steps:
                return out
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--every", type=int, default=20)
    ap.add_argument("--variants", default="native,torch,loss_torch,optim_torch,unfused,model_torch,aug_torch")
    ap.add_argument("--seeds", default="0")
    a = ap.parse_args()
    for seed in [int(s) for s in a.seeds.split(",")]:
      for v in a.variants.split(","):
        torch.manual_seed(seed)
        try:
            r = run(v, a.steps, a.every, seed)
            print(f"{v:12s} s{seed} " + "  ".join(f"{s}:{l}({nm})" for s, l, nm in r), flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{v:12s} FAILED {e!r}", flush=True)


if __name__ == "__main__":
    main()
