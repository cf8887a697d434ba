#!/usr/bin/env python3
"""Loss trajectories of native bf16 vs fp32 torch vs torch bf16 autocast on the same
augmented views (SimCLR, class-structured synthetic CIFAR-shaped data).

python tools/trajectory_probe.py [model] [steps] [lr] [batch]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    lr0 = float(sys.argv[3]) if len(sys.argv) > 3 else 0.1
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    from simclr_pytorch_distributed_amd.data.augment import AugConfig, gpu_augment, nhwc8_to_nchw
    from simclr_pytorch_distributed_amd.data.datasets import build_dataset
    from simclr_pytorch_distributed_amd.losses.supcon import DistributedContrastiveLoss
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams, FusedSGD
    gpu = torch.device("cuda:0")
    torch.manual_seed(0)
    a = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last)
    b = SupConResNet(name).to(gpu)
    c = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last)
    b.load_state_dict(a.state_dict())
    c.load_state_dict(a.state_dict())
    flat = FlatParams(a)
    r = ModelRunner(a, "native", master=flat.flat)
    on = FusedSGD(flat, lr=lr0, momentum=0.9, weight_decay=1e-4)
    ob = torch.optim.SGD(b.parameters(), lr=lr0, momentum=0.9, weight_decay=1e-4)
    oc = torch.optim.SGD(c.parameters(), lr=lr0, momentum=0.9, weight_decay=1e-4)
    cn = DistributedContrastiveLoss("SimCLR", 0.5, backend="native")
    ct = DistributedContrastiveLoss("SimCLR", 0.5, backend="torch")
    ds = build_dataset("cifar10", None, True, True, 4096, 32, 0)
    data = torch.from_numpy(ds.images).to(gpu)
    aug = AugConfig.simclr(32, (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))
    rows = []
    for step in range(steps):
        lr = lr0 * min(1.0, (step + 1) / 10)
        on.param_groups[0]["lr"] = lr
        for o in (ob, oc):
            for gp in o.param_groups:
                gp["lr"] = lr
        idx = torch.arange(B * step, B * step + B, device=gpu) % data.shape[0]
        v = gpu_augment(data, idx, aug, 1000 + step)
        vt = nhwc8_to_nchw(v)
        on.zero_grad()
        ln = cn(r.forward(v))
        ln.backward()
        on.step()
        ob.zero_grad()
        lt = ct(b(vt))
        lt.backward()
        ob.step()
        oc.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lc = ct(c(vt).float())
        lc.backward()
        oc.step()
        rows.append((float(ln.detach()), float(lt.detach()), float(lc.detach())))
    torch.cuda.synchronize()
    print(f"{name} lr {lr0} batch {B}: step  native  fp32  autocast")
    for s in list(range(0, steps, 5)) + [steps - 1]:
        n_, t_, c_ = rows[s]
        print(f"  {s:4d} {n_:9.4f} {t_:9.4f} {c_:9.4f}   dn {abs(n_ - t_) / t_:.3%}  dc {abs(c_ - t_) / t_:.3%}")


if __name__ == "__main__":
    main()
