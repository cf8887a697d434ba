#!/usr/bin/env python3
"""Localise native-vs-fp32 gradient differences: per-parameter rel/cos for a linear
functional of the head output (ResNet-50, 32 views), for several executor variants.

python tools/grad_parity_probe.py [resnet50|resnet18] [fused|unfused]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    fused = (sys.argv[2] if len(sys.argv) > 2 else "fused") == "fused"
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner, to_nhwc_input
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    gpu = torch.device("cuda:0")
    torch.manual_seed(0)
    a = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last)
    b = SupConResNet(name).to(gpu)
    b.load_state_dict(a.state_dict())
    flat = FlatParams(a)
    r = ModelRunner(a, "native", master=flat.flat, fused=fused)
    x = torch.randn(32, 3, 32, 32, generator=torch.Generator().manual_seed(1)).to(gpu).to(torch.bfloat16).float()
    G = torch.randn(32, 128, generator=torch.Generator().manual_seed(3)).to(gpu)
    flat.zero_grad()
    on = r.forward(to_nhwc_input(x))
    (on * G).sum().backward()
    torch.cuda.synchronize()
    ot = b(x)
    (ot * G).sum().backward()
    print(f"{name} fused={fused} out rel {float((on - ot).norm() / ot.norm()):.4g}")
    # control: the same model in torch bf16 autocast (MIOpen / hipBLASLt) vs fp32
    c = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last)
    c.load_state_dict(b.state_dict())
    with torch.autocast("cuda", dtype=torch.bfloat16):
        oc = c(x).float()
    (oc * G).sum().backward()
    print(f"torch-bf16 autocast out rel {float((oc - ot).norm() / ot.norm()):.4g}")
    for (n, p), (_, q), (_, k) in zip(a.named_parameters(), b.named_parameters(), c.named_parameters()):
        gt = q.grad.double().flatten()
        res = []
        for g in (p.grad, k.grad):
            g = g.double().flatten()
            res.append((float((g - gt).norm() / (gt.norm() + 1e-30)), float(torch.dot(g, gt) / (g.norm() * gt.norm() + 1e-30))))
        print(f"  {n:45s} native rel {res[0][0]:8.4g} cos {res[0][1]:8.5f} | autocast rel {res[1][0]:8.4g} cos {res[1][1]:8.5f}")


if __name__ == "__main__":
    main()
