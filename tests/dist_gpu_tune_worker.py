"""Worker for tests/test_gpu_dist.py::test_syncbn_autotune_agrees: builds the pretrain
engine with --syncbn_comm auto as rank RANK of WORLD_SIZE (gloo process group, every rank on
cuda:0) and runs the SyncBN transport measurement on one batch. Writes the choice, the
reduced timings and whether the training state came back unchanged to OUT_DIR."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    out_dir = sys.argv[1]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    argv = ["--model", "resnet18", "--backend", "native", "--dist_backend", "gloo", "--synthetic",
            "--synthetic_size", "64", "--learning_rate", "0.05", "--work_dir", out_dir, "--batch_size", "32",
            "--ngpu", str(world), "--syncBN", "--syncbn_comm", "auto"]
    opt = parse_pretrain(argv, make_dirs=False)
    eng = PretrainEngine(opt, device=torch.device("cuda:0"))
    eng.sampler.set_epoch(1)
    idx = next(eng.sampler.batches(eng.device))
    before = eng.flat.flat.detach().clone()
    bufs = [b.detach().clone() for b in eng.model.buffers()]
    tune = eng.autotune_syncbn(idx, steps=1, baseline=True)
    torch.cuda.synchronize()
    restored = torch.equal(before, eng.flat.flat) and all(torch.equal(a, b) for a, b in zip(bufs, eng.model.buffers()))
    with open(os.path.join(out_dir, f"tune_r{rank}.json"), "w") as f:
        json.dump({"tune": tune, "transport": eng.syncbn_transport, "restored": restored}, f)
    import torch.distributed as dist
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
