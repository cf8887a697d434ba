#!/usr/bin/env python3
"""BN3 fold precision probe at the headline batch: blocks l1.1 -> l1.2 (and l2.1 -> l2.2)
teacher-forced at 512 views, BN-parameter gradients of the native path with the fold on /
off and of torch bf16 autocast, each vs fp32 torch (same bf16 input, same bf16 upstream
gradient). Prints rel errors per BN parameter."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.models.executor import ModelRunner
from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
from simclr_pytorch_distributed_amd.ops import block as fb
from simclr_pytorch_distributed_amd.optim.flat import FlatParams


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    nat = SupConResNet("resnet50").to(dev).to(memory_format=torch.channels_last)
    ref = SupConResNet("resnet50").to(dev)
    ref.load_state_dict(nat.state_dict())
    flat = FlatParams(nat)
    runner = ModelRunner(nat, "native", master=flat.flat)
    wc = runner.weight_cache()
    nb, rb = list(nat.encoder.blocks()), list(ref.encoder.blocks())
    g = torch.Generator().manual_seed(3)
    views = int(os.environ.get("VIEWS", "512"))
    for i, hw in ((1, 32), (4, 16)):
        c_in = nb[i].conv1.in_channels
        x = torch.randn(views, c_in, hw, hw, generator=g).relu().to(dev).to(torch.bfloat16).float()
        res = {}
        dy = None
        for fold in (False, True):
            fb.BN3_FOLD = fold
            flat.zero_grad()
            wc.refresh()
            chain = fb.BlockChain()
            xn = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).requires_grad_(True)
            out = fb.bottleneck(fb.bottleneck(xn, nb[i], wc, True, None, chain), nb[i + 1], wc, True, None, chain)
            if dy is None:
                dy = torch.randn(out.shape, generator=g).to(dev).to(torch.bfloat16)
            out.backward(dy)
            torch.cuda.synchronize()
            res[fold] = {n: p.grad.float().clone() for j in (i, i + 1) for n, p in
                         [(f"b{j}.{n}", p) for n, p in nb[j].named_parameters()]}
        dyt = dy.float().permute(0, 3, 1, 2)
        for blk in rb[i:i + 2]:
            blk.zero_grad()
        xt = x.clone().requires_grad_(True)
        rb[i + 1](rb[i](xt)).backward(dyt)
        truth = {f"b{j}.{n}": p.grad.float() for j in (i, i + 1) for n, p in rb[j].named_parameters()}
        cb = [copy.deepcopy(rb[j]).to(memory_format=torch.channels_last) for j in (i, i + 1)]
        for blk in cb:
            blk.zero_grad()
        xc = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            oc = cb[1](cb[0](xc)).float()
        oc.backward(dyt)
        auto = {f"b{j}.{n}": p.grad.float() for k, j in enumerate((i, i + 1)) for n, p in cb[k].named_parameters()}
        print(f"pair {i},{i + 1} at {views} views: rel error vs fp32 (unfolded / fold / autocast)")
        for n in truth:
            if "bn" in n or "conv3" in n:
                print(f"  {n:24s} {rel(res[False][n], truth[n]):.4f} {rel(res[True][n], truth[n]):.4f} "
                      f"{rel(auto[n], truth[n]):.4f}", flush=True)


if __name__ == "__main__":
    main()
