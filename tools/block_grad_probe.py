#!/usr/bin/env python3
"""Teacher-forced backward of single blocks / block pairs: native executor, native
per-op path and torch bf16 autocast vs fp32 torch (same bf16 input and upstream grad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.models.resnet import Bottleneck, SupConResNet
    from simclr_pytorch_distributed_amd.ops import block as fb
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    gpu = torch.device("cuda:0")
    torch.manual_seed(0)
    a = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last)
    b = SupConResNet(name).to(gpu)
    b.load_state_dict(a.state_dict())
    flat = FlatParams(a)
    runner = ModelRunner(a, "native", master=flat.flat)
    wc = runner.weight_cache()
    nb, rb = list(a.encoder.blocks()), list(b.encoder.blocks())
    g = torch.Generator().manual_seed(9)
    x0 = torch.randn(32, 3, 32, 32, generator=torch.Generator().manual_seed(1)).to(gpu)
    with torch.no_grad():
        r = torch.relu(b.encoder.bn1(b.encoder.conv1(x0)))
    for i in range(min(4, len(nb))):
        xin = r.to(torch.bfloat16).float()
        for mode in ("single", "native_exec_off"):
            os.environ["X"] = "1"
            old = fb.NATIVE_EXEC
            fb.NATIVE_EXEC = mode == "single"
            flat.zero_grad()
            wc.refresh()
            xn = xin.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).requires_grad_(True)
            blk = nb[i]
            out = (fb.bottleneck if isinstance(blk, Bottleneck) else fb.basic)(xn, blk, wc, True, None, None)
            dy = torch.randn(out.shape, generator=torch.Generator().manual_seed(100 + i)).to(gpu).to(torch.bfloat16)
            out.backward(dy)
            torch.cuda.synchronize()
            fb.NATIVE_EXEC = old
            xt = xin.clone().requires_grad_(True)
            rb[i].zero_grad()
            ot = rb[i](xt)
            ot.backward(dy.float().permute(0, 3, 1, 2))
            fo = rel(out.float().permute(0, 3, 1, 2), ot)
            print(f"block {i} {mode:16s} out {fo:.4f} dx {rel(xn.grad.float().permute(0, 3, 1, 2), xt.grad):.4f} "
                  + " ".join(f"{n}:{rel(p.grad, q.grad):.4f}" for (n, p), (_, q) in
                             zip(nb[i].named_parameters(), rb[i].named_parameters())))
        # autocast control
        c = type(rb[i])  # same module class
        import copy
        cb = copy.deepcopy(rb[i]).to(memory_format=torch.channels_last)
        cb.zero_grad()
        xc = xin.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            oc = cb(xc).float()
        oc.backward(dy.float().permute(0, 3, 1, 2))
        print(f"block {i} {'autocast':16s} out {rel(oc, ot):.4f} dx {rel(xc.grad, xt.grad):.4f} "
              + " ".join(f"{n}:{rel(p.grad, q.grad):.4f}" for (n, p), (_, q) in
                         zip(cb.named_parameters(), rb[i].named_parameters())))
        with torch.no_grad():
            r = rb[i](xin)


if __name__ == "__main__":
    main()
