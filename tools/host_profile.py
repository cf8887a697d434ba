#!/usr/bin/env python3
"""cProfile of the host side of the native training step (where do the milliseconds of
Python / launch overhead per step go?); 20 steps, sorted by own time and by cumulative time."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import logging
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    logging.disable(logging.INFO)
    bs = os.environ.get("HP_BS", "256")          # HP_BS: images per step; HP_SYNC=1: idle queue
    sync = os.environ.get("HP_SYNC", "0") == "1"  # (sync after each step: pure host cost)
    opt = parse_pretrain(["--batch_size", bs, "--synthetic", "--synthetic_size", "8192", "--backend", "native",
                          "--work_dir", "/tmp/hp", "--temp", "0.5", "--cosine"], make_dirs=False)
    eng = PretrainEngine(opt)
    eng.model.train()
    eng.sampler.set_epoch(1)
    idxs = list(eng.sampler.batches(eng.device))
    for i in range(5):
        eng.train_step(idxs[i], 1, i, len(idxs))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for i in range(20):
        eng.train_step(idxs[5 + i], 1, 5 + i, len(idxs))
        if sync:
            torch.cuda.synchronize()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(40)
    st.sort_stats("cumulative").print_stats(60)


if __name__ == "__main__":
    main()
