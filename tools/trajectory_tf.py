#!/usr/bin/env python3
"""Teacher-forced gradient parity along an fp32 training trajectory.

The fp32 torch model (reference math: networks/resnet_big.py, losses.py,
main_supcon.py:266-325) takes the SGD steps. Before every step its parameters and BN
buffers are copied into the native model and into a torch bf16-autocast control, and all
three compute the gradient of the SimCLR loss on the SAME augmented views. Per step it
prints, for native and autocast vs fp32: the loss gap, the global gradient-norm ratio,
the global cosine, and the relative error per stage (stem, layer1..4, head).

A systematic native gradient bias shows up as a native column that is worse than the
autocast column step after step; chaotic divergence of free-running trajectories does
not (both columns stay small while the free runs separate).

``free`` mode instead runs the trajectories independently and logs loss + global gradient
norm per step (the free-running probe with gradient norms), with a SECOND fp32 replica from
the same initial weights on the same views: torch's GPU kernels are not bit-deterministic,
so the fp32-vs-fp32 gap is the chaos floor of the trajectory itself.

python tools/trajectory_tf.py [tf|free] [model] [steps] [lr] [batch]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

STAGES = ("stem", "layer1", "layer2", "layer3", "layer4", "head")


def _stage(name):
    for s in STAGES[1:]:
        if f".{s}." in f".{name}" or name.startswith(s):
            return s
    return "stem"


def _gvec(model):
    return torch.cat([p.grad.detach().double().flatten() for p in model.parameters()])


def _groups(model):
    out, off = {}, 0
    for n, p in model.named_parameters():
        k = p.numel()
        out.setdefault(_stage(n), []).append((off, off + k))
        off += k
    return out


def _cmp(g, gt, groups):
    rel = float((g - gt).norm() / (gt.norm() + 1e-30))
    cos = float(torch.dot(g, gt) / (g.norm() * gt.norm() + 1e-30))
    ratio = float(g.norm() / (gt.norm() + 1e-30))
    per = {}
    for s, spans in groups.items():
        a = torch.cat([g[i:j] for i, j in spans])
        b = torch.cat([gt[i:j] for i, j in spans])
        per[s] = float((a - b).norm() / (b.norm() + 1e-30))
    return rel, cos, ratio, per


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "tf"
    name = sys.argv[2] if len(sys.argv) > 2 else "resnet50"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    lr0 = float(sys.argv[4]) if len(sys.argv) > 4 else 0.05
    B = int(sys.argv[5]) if len(sys.argv) > 5 else 128
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
    d = SupConResNet(name).to(gpu) if mode == "free" else None
    b.load_state_dict(a.state_dict())
    c.load_state_dict(a.state_dict())
    if d is not None:
        d.load_state_dict(a.state_dict())
    flat = FlatParams(a)
    r = ModelRunner(a, "native", master=flat.flat)
    on = FusedSGD(flat, lr=lr0, momentum=0.9, weight_decay=1e-4)
    ob = torch.optim.SGD(b.parameters(), lr=lr0, momentum=0.9, weight_decay=1e-4)
    oc = torch.optim.SGD(c.parameters(), lr=lr0, momentum=0.9, weight_decay=1e-4)
    od = torch.optim.SGD(d.parameters(), lr=lr0, momentum=0.9, weight_decay=1e-4) if d is not None else None
    cn = DistributedContrastiveLoss("SimCLR", 0.5, backend="native")
    ct = DistributedContrastiveLoss("SimCLR", 0.5, backend="torch")
    ds = build_dataset("cifar10", None, True, True, 4096, 32, 0)
    data = torch.from_numpy(ds.images).to(gpu)
    aug = AugConfig.simclr(32, (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))
    groups = _groups(b)
    env = {k: v for k, v in os.environ.items() if k.startswith("SDX_")}
    print(f"{mode} {name} lr {lr0} batch {B} steps {steps} env {env}", flush=True)
    if mode == "tf":
        print("step  loss_fp32  dloss_nat  dloss_ac | rel_nat rel_ac | cos_nat cos_ac | |g|nat/fp32 |g|ac/fp32 | "
              "per-stage rel nat/ac " + " ".join(STAGES), flush=True)
    else:
        print("step  loss: native fp32 autocast fp32-replica | |g|: native fp32 autocast", flush=True)
    acc = {"n": [], "c": []}
    for step in range(steps):
        lr = lr0 * min(1.0, (step + 1) / 10)
        on.param_groups[0]["lr"] = lr
        for o in (ob, oc, od):
            if o is None:
                continue
            for gp in o.param_groups:
                gp["lr"] = lr
        if mode == "tf":
            with torch.no_grad():
                sd = b.state_dict()
                a.load_state_dict(sd)
                c.load_state_dict(sd)
        idx = torch.arange(B * step, B * step + B, device=gpu) % data.shape[0]
        v = gpu_augment(data, idx, aug, 1000 + step)
        vt = nhwc8_to_nchw(v)
        on.zero_grad()
        ln = cn(r.forward(v))
        ln.backward()
        ob.zero_grad()
        lt = ct(b(vt))
        lt.backward()
        oc.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lc = ct(c(vt).float())
        lc.backward()
        ld = None
        if d is not None:
            od.zero_grad()
            ld = ct(d(vt))
            ld.backward()
        torch.cuda.synchronize()
        gn, gt, gc = _gvec(a), _gvec(b), _gvec(c)
        if mode == "tf":
            rn, cosn, qn, pn = _cmp(gn, gt, groups)
            rc, cosc, qc, pc = _cmp(gc, gt, groups)
            acc["n"].append(rn)
            acc["c"].append(rc)
            lt_ = float(lt.detach())
            print(f"{step:4d} {lt_:9.4f} {float(ln.detach()) - lt_:+9.5f} {float(lc.detach()) - lt_:+9.5f} | {rn:.4f} {rc:.4f} | "
                  f"{cosn:.5f} {cosc:.5f} | {qn:.4f} {qc:.4f} | "
                  + " ".join(f"{pn[s]:.3f}/{pc[s]:.3f}" for s in STAGES), flush=True)
            ob.step()
        else:
            on.step()
            ob.step()
            oc.step()
            od.step()
            print(f"{step:4d} {float(ln.detach()):9.4f} {float(lt.detach()):9.4f} {float(lc.detach()):9.4f} {float(ld.detach()):9.4f} | "
                  f"{float(gn.norm()):.4e} {float(gt.norm()):.4e} {float(gc.norm()):.4e}", flush=True)
    if mode == "tf":
        mn = sum(acc["n"]) / len(acc["n"])
        mc = sum(acc["c"]) / len(acc["c"])
        print(f"mean global grad rel err vs fp32: native {mn:.4f}  autocast {mc:.4f}  ratio {mn / max(mc, 1e-12):.3f}")


if __name__ == "__main__":
    main()
