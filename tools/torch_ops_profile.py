#!/usr/bin/env python3
"""Host-side attribution of the small torch ops in one native training step (torch.profiler):
which aten ops (copies, fills, casts) run per step and from where.

python tools/torch_ops_profile.py
"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile


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
    for i in range(4):
        eng.train_step(next(it), 1, i, 100)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        eng.train_step(next(it), 1, 5, 100)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=4)
    rows = [e for e in ka if e.key.startswith("aten::") and e.key in
            ("aten::copy_", "aten::fill_", "aten::zero_", "aten::to", "aten::_to_copy", "aten::clone", "aten::cat",
             "aten::contiguous", "aten::add_", "aten::mul", "aten::add", "aten::sum", "aten::norm", "aten::item",
             "aten::_local_scalar_dense", "aten::empty", "aten::zeros", "aten::where", "aten::div")]
    rows.sort(key=lambda e: -e.count)
    for e in rows[:40]:
        st = " <- ".join(s.split("/")[-1] for s in (e.stack or [])[:4])
        print(f"{e.count:4d} {e.key:28s} {e.cpu_time_total / 1e3:8.2f} ms  {st}")
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25))


if __name__ == "__main__":
    main()
