#!/usr/bin/env python3
"""Host-side (no GPU sync) time per phase of the native training step, steady state.

python tools/host_phases.py [--steps 20]
"""
import os
import sys
import tempfile
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    import logging
    logging.disable(logging.INFO)
    opt = parse_pretrain(["--batch_size", "256", "--synthetic", "--synthetic_size", "8192", "--cosine",
                          "--learning_rate", "0.5", "--temp", "0.5", "--work_dir", tempfile.mkdtemp()],
                         make_dirs=False)
    eng = PretrainEngine(opt)
    eng.model.train()
    eng.sampler.set_epoch(1)
    it = eng.sampler.batches(eng.device)
    T = defaultdict(float)
    n = 0
    for i in range(25):
        idx = next(it)
        t = [time.perf_counter()]
        eng._host_prelude(1, i, 100)
        x = eng.make_views(idx, 1, i)
        t.append(time.perf_counter())
        feats = eng.runner.forward(x)
        t.append(time.perf_counter())
        loss = eng.criterion(feats, None)
        t.append(time.perf_counter())
        stats = eng._norm_terms(feats)
        ex = stats.pop("extra_loss")
        loss = loss if ex is None else loss + ex
        t.append(time.perf_counter())
        eng.optimizer.zero_grad()
        loss.backward()
        t.append(time.perf_counter())
        eng.optimizer.step()
        t.append(time.perf_counter())
        if i >= 5:
            n += 1
            for k, name in enumerate(["prelude+aug", "forward", "loss", "norm_terms", "backward", "optimizer"]):
                T[name] += (t[k + 1] - t[k]) * 1e3
    torch.cuda.synchronize()
    tot = sum(T.values()) / n
    for k, v in T.items():
        print(f"{k:12s} {v / n:7.3f} ms")
    print(f"{'total':12s} {tot:7.3f} ms (host, steady state, no sync)")
    # idle-queue host cost: sync before each phase
    T2 = defaultdict(float)
    it = eng.sampler.batches(eng.device)
    for i in range(8):
        idx = next(it)
        torch.cuda.synchronize(); a = time.perf_counter()
        feats = eng.runner.forward(eng.make_views(idx, 1, i)); b = time.perf_counter()
        torch.cuda.synchronize(); b2 = time.perf_counter()
        loss = eng.criterion(feats, None); st = eng._norm_terms(feats); ex = st.pop("extra_loss"); loss = loss if ex is None else loss + ex
        c = time.perf_counter()
        torch.cuda.synchronize(); c2 = time.perf_counter()
        eng.optimizer.zero_grad(); loss.backward(); d = time.perf_counter()
        torch.cuda.synchronize(); d2 = time.perf_counter()
        eng.optimizer.step(); e = time.perf_counter()
        torch.cuda.synchronize(); e2 = time.perf_counter()
        if i >= 3:
            for k, v in (("fwd host", b - a), ("fwd gpu+host", b2 - a), ("loss host", c - b2), ("loss gpu+host", c2 - b2),
                         ("bwd host", d - c2), ("bwd gpu+host", d2 - c2), ("opt host", e - d2), ("opt gpu+host", e2 - d2)):
                T2[k] += v * 1e3 / 5
    for k, v in T2.items():
        print(f"{k:14s} {v:7.3f} ms (idle queue)")


if __name__ == "__main__":
    main()
