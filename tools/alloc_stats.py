#!/usr/bin/env python3
"""Caching-allocator activity per steady-state training step (device allocs/frees, retries,
stream syncs): any nonzero per-step hipMalloc/hipFree means a hidden device sync.

python tools/alloc_stats.py
"""
import os
import sys
import tempfile

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
    keys = ["num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams", "num_ooms"]
    for i in range(20):
        if i == 10:
            torch.cuda.synchronize()
            s0 = torch.cuda.memory_stats()
        eng.train_step(next(it), 1, i, 100)
    torch.cuda.synchronize()
    s1 = torch.cuda.memory_stats()
    for k in keys:
        print(f"{k:24s} per step over 10 steps: {(s1.get(k, 0) - s0.get(k, 0)) / 10:.2f}")
    from collections import Counter
    segs = torch.cuda.memory_snapshot()
    c = Counter()
    for sg in segs:
        c[(sg["stream"], sg["segment_type"], sg["total_size"] >> 20)] += 1
    for (st, ty, mb), n in sorted(c.items(), key=lambda kv: -kv[0][2] * kv[1])[:15]:
        act = sum(b["size"] for sg in segs if sg["stream"] == st and sg["total_size"] >> 20 == mb
                  for b in sg["blocks"] if b["state"] == "active_allocated") >> 20
        print(f"stream {st:#x} {ty:6s} {mb:7d} MiB x {n}  (active MiB in these: {act})")
    print(f"reserved {s1['reserved_bytes.all.current'] / 2**30:.2f} GiB, peak allocated "
          f"{s1['allocated_bytes.all.peak'] / 2**30:.2f} GiB")


if __name__ == "__main__":
    main()
