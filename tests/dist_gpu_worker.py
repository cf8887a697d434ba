"""Worker for tests/test_gpu_dist.py: one native training step on cuda:0 as rank RANK of
WORLD_SIZE (gloo carries the collectives, so several ranks can share the one GPU of the
test box). Writes the updated flat parameters and BN running stats to OUT_DIR."""
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
    from simclr_pytorch_distributed_amd.models.executor import to_nhwc_input
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    from simclr_pytorch_distributed_amd.parallel import comm
    name = os.environ.get("SDX_TEST_MODEL", "resnet18")
    G = 32                                    # global images (16 per rank at W=2: 32 views, so
    #                                           ResNet-50 layer 1 folds its BN3 on every rank)
    argv = ["--model", name, "--backend", os.environ.get("SDX_TEST_BACKEND", "native"), "--dist_backend", "gloo", "--synthetic",
            "--synthetic_size", "64", "--learning_rate", "0.05", "--grad_semantics", "exact",
            "--work_dir", out_dir, "--batch_size", str(G), "--ngpu", str(world)]
    if os.environ.get("SDX_TEST_GRAD_COMPRESS"):
        argv += ["--grad_compress", os.environ["SDX_TEST_GRAD_COMPRESS"]]
    if world > 1:
        argv.append("--syncBN")
        # '' = rccl, which over the gloo process group means the Python collective path
        argv += ["--syncbn_comm", os.environ.get("SDX_TEST_SYNCBN_COMM") or "rccl"]
    opt = parse_pretrain(argv, make_dirs=False)
    eng = PretrainEngine(opt, device=torch.device("cuda:0"))
    torch.manual_seed(123)
    init = SupConResNet(name).state_dict()
    eng.model.load_state_dict(init)
    eng.model.train()
    g = torch.Generator().manual_seed(7)
    imgs = torch.randn(2, G, 3, 32, 32, generator=g)          # [view][global batch]
    per = G // world
    sl = slice(rank * per, (rank + 1) * per)
    x = torch.cat([imgs[0, sl], imgs[1, sl]]).cuda()
    feats = eng.runner.forward(to_nhwc_input(x) if eng.backend == "native" else x)
    loss = eng.criterion(feats)
    eng.optimizer.zero_grad()
    loss.backward()
    if eng.reducer is not None:
        eng.reducer.finish()
    grad = eng.flat.grad.detach().clone()
    eng.optimizer.step()
    torch.cuda.synchronize()

    def state_hash():
        # exact replica fingerprint: every parameter and every BN running statistic, bit for bit
        flat = eng.flat.flat.detach().view(torch.int32).to(torch.int64)
        bufs = [b.detach().reshape(-1).float().view(torch.int32).to(torch.int64) for b in eng.model.buffers()
                if b.is_floating_point()]
        w = torch.arange(1, flat.numel() + 1, device=flat.device, dtype=torch.int64)
        hf = int((flat * w).sum()) & ((1 << 62) - 1)
        hb = int(sum(int((t * torch.arange(1, t.numel() + 1, device=t.device, dtype=torch.int64)).sum()) for t in bufs))
        return hf, hb & ((1 << 62) - 1)

    hashes = [state_hash()]
    # SDX_TEST_STEPS > 1: further steps on fresh data (replicas and running statistics must stay
    # bit-identical across ranks after every step; >300 SyncBN exchanges at ResNet-50 x 3 steps)
    for step in range(1, int(os.environ.get("SDX_TEST_STEPS", "1"))):
        gs = torch.Generator().manual_seed(7 + step)
        im = torch.randn(2, G, 3, 32, 32, generator=gs)
        xs = torch.cat([im[0, sl], im[1, sl]]).cuda()
        fs = eng.runner.forward(to_nhwc_input(xs) if eng.backend == "native" else xs)
        ls = eng.criterion(fs)
        eng.optimizer.zero_grad()
        ls.backward()
        if eng.reducer is not None:
            eng.reducer.finish()
        eng.optimizer.step()
        torch.cuda.synchronize()
        hashes.append(state_hash())
    bn = eng.model.encoder.layer1[0].bn1
    torch.save({"hashes": hashes, "flat": eng.flat.flat.detach().cpu() if len(hashes) == 1 else None,
                "rm": bn.running_mean.cpu(), "rv": bn.running_var.cpu(),
                "native_h": comm.native_small_comm(None), "loss": float(loss.detach()), "grad": grad.cpu(), "names": list(eng.flat.names),
                "offsets": [int(o) for o in eng.flat.offsets], "numels": [p.numel() for p in eng.flat.params]}, os.path.join(out_dir, f"{name}_w{world}{os.environ.get('SDX_TEST_GRAD_COMPRESS', '')}_r{rank}.pt"))
    print(f"rank {rank}: state hashes per step {hashes}")
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
