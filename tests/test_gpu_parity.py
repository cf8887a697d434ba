"""Whole-network parity of the native bf16 training path against fp32 torch autograd
(reference math: networks/resnet_big.py, losses.py, main_supcon.py:266-325).

* gradient parity, two ways: (a) the whole ResNet-50 + MLP head through the fused
  native executor (implicit-GEMM convs, BN statistics from conv and dgrad epilogues,
  compact shortcut gradients, ReLU bitmasks, fused head) vs plain fp32 torch autograd
  on the same bf16-rounded images, with torch's own bf16 autocast path as the bar (at
  random init bf16 rounding alone moves this network's output by ~13 %); (b) every pair
  of consecutive blocks teacher-forced, with an absolute bar (cos >= 0.999, rel <= 2e-2)
  on every parameter and the input gradient.
* trajectory parity: 50 SGD steps (lr 0.05, momentum 0.9, 10-step warm-up ramp, SimCLR
  tau 0.5) on augmented class-structured synthetic images — the native bf16 loss must
  track the fp32 torch loss (10-step window means within 2.5 %), and both must fall.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(gpu, name="resnet50"):
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    torch.manual_seed(0)
    a = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last)
    b = SupConResNet(name).to(gpu)
    b.load_state_dict(a.state_dict())
    return a, b


def _images(gpu, n, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, 3, 32, 32, generator=g).to(gpu)
    return x.to(torch.bfloat16).float()          # both paths see the same bf16 values


def _grad_rows(ref_model, *models):
    """Per parameter: (name, [(rel, cos) of each model's gradient vs ref_model's])."""
    out = []
    named = [list(m.named_parameters()) for m in models]
    for i, (n, q) in enumerate(ref_model.named_parameters()):
        gt = q.grad.double().flatten()
        res = []
        for nm in named:
            g = nm[i][1].grad.double().flatten()
            res.append((float((g - gt).norm() / (gt.norm() + 1e-30)),
                        float(torch.dot(g, gt) / (g.norm() * gt.norm() + 1e-30))))
        out.append((n, res))
    return out


def _autocast_copy(gpu, ref_m):
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    name = "resnet50" if hasattr(ref_m.encoder.layer1[0], "conv3") else "resnet18"
    c = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last)
    c.load_state_dict(ref_m.state_dict())
    return c


@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
def test_whole_network_gradients_within_bf16_envelope(gpu, name):
    """Whole network, 32 views, loss = <head output, G> (fixed random G: an O(1),
    well-conditioned feature gradient), native executor vs fp32 torch autograd on the same
    bf16-rounded images. The bar is torch's own bf16 autocast path (MIOpen / hipBLASLt):
    bf16 rounding flips ReLU masks, and at random init those flips compound through the
    depth (ResNet-50's output moves ~13 % under ANY bf16 path, measured native 12.8 %,
    autocast 13.3 %: tools/grad_parity_probe.py), so an absolute fp32 bar is unreachable
    there. ResNet-18 (≈1.3 % output change): every one of its parameter gradients must be
    about as close to fp32 as autocast's (rel <= 1.5x autocast + 0.02, cos >= autocast -
    0.05; measured worst: the stem / first-block BN parameters, where the compounded
    mask-flip noise of 8 blocks lands, at 1.2-1.3x — block by block the native errors are
    within 1.2x autocast, test_block_pairs_gradients_match_fp32).
    ResNet-50: the output and the head gradients, which are still well conditioned."""
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner, to_nhwc_input
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    nat_m, ref_m = _models(gpu, name)
    ctl_m = _autocast_copy(gpu, ref_m)
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    x = _images(gpu, 32)
    G = torch.randn(32, 128, generator=torch.Generator().manual_seed(3)).to(gpu)
    flat.zero_grad()
    on = runner.forward(to_nhwc_input(x))
    (on * G).sum().backward()
    torch.cuda.synchronize()
    ot = ref_m(x)
    (ot * G).sum().backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        oc = ctl_m(x).float()
    (oc * G).sum().backward()
    e_n = float((on - ot).norm() / ot.norm())
    e_c = float((oc - ot).norm() / ot.norm())
    print(f"{name} output rel error: native {e_n:.4g}, autocast {e_c:.4g}")
    assert e_n <= 1.2 * e_c + 1e-3
    rows = _grad_rows(ref_m, nat_m, ctl_m)
    assert len(rows) == len(list(ref_m.parameters()))
    if name == "resnet50":
        rows = [r for r in rows if r[0].startswith("head")]
    bad = [(n, r) for n, r in rows if not (r[0][0] <= 1.5 * r[1][0] + 0.02 and r[0][1] >= r[1][1] - 0.05)]
    worst = sorted(rows, key=lambda t: t[1][0][0] - t[1][1][0], reverse=True)[:4]
    print("largest native-minus-autocast rel errors:",
          "; ".join(f"{n}: {r[0][0]:.3g} vs {r[1][0]:.3g}" for n, r in worst))
    assert not bad, f"{len(bad)} of {len(rows)} gradients outside the bf16 envelope: {bad[:6]}"


@pytest.mark.parametrize("name,fold", [("resnet50", False), ("resnet50", True), ("resnet18", False)])
def test_block_pairs_gradients_match_fp32(gpu, name, fold, monkeypatch):
    """Teacher-forced backward of every pair of consecutive residual blocks through the
    native executor (so the cross-block hand-off of BN-backward sums from the next
    block's final dgrad epilogue, the compact strided-shortcut gradient and the ReLU
    bitmasks are all exercised) vs the same two blocks in fp32 torch, on the same
    bf16-rounded input and bf16 upstream gradient. A random upstream gradient makes every
    ReLU mask flip of bf16 rounding count in full (≈5-8 % relative error for ANY bf16
    path, measured with torch autocast: tools/block_grad_probe.py), so the bar per
    parameter and for the input gradient is the autocast error of the same pair:
    rel <= 1.2x autocast + 0.01 and cos >= autocast cos - 0.005."""
    import copy
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.models.resnet import Bottleneck
    from simclr_pytorch_distributed_amd.ops import block as fb
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    # fold: identity bottlenecks of layers 1-2 with the BN3 fold (csrc/kernels/bnfold.hip);
    # pairs (2,3), (4,5), (6,7) have a folding first block
    monkeypatch.setattr(fb, "BN3_FOLD", fold)
    monkeypatch.setattr(fb, "BN3_FOLD_ROWS_PER_K2", 0.0)   # fold at this small batch too
    monkeypatch.setattr(fb, "BN3_FOLD_MAXK", 128)
    nat_m, ref_m = _models(gpu, name)
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    wc = runner.weight_cache()
    nb, rb = list(nat_m.encoder.blocks()), list(ref_m.encoder.blocks())
    g = torch.Generator().manual_seed(9)
    with torch.no_grad():
        r = torch.relu(ref_m.encoder.bn1(ref_m.encoder.conv1(_images(gpu, 32))))

    def score(a, b):
        a, b = a.double().flatten(), b.double().flatten()
        return float((a - b).norm() / (b.norm() + 1e-30)), float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))

    failures, worst = [], (0.0, "")
    for i in range(0, len(nb) - 1, 2):
        xin = r.to(torch.bfloat16).float().detach()
        flat.zero_grad()
        wc.refresh()
        chain = fb.BlockChain()
        xn = xin.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).requires_grad_(True)
        out = xn
        for j, blk in enumerate(nb[i:i + 2]):
            out = fb.bottleneck(out, blk, wc, True, None, chain, next_native=j == 0) if isinstance(blk, Bottleneck) \
                else fb.basic(out, blk, wc, True, None, chain)
        dy = torch.randn(out.shape, generator=g).to(gpu).to(torch.bfloat16)
        out.backward(dy)
        torch.cuda.synchronize()
        dyt = dy.float().permute(0, 3, 1, 2)
        xt = xin.clone().requires_grad_(True)
        for blk in rb[i:i + 2]:
            blk.zero_grad()
        rb[i + 1](rb[i](xt)).backward(dyt)
        cb = [copy.deepcopy(rb[j]).to(memory_format=torch.channels_last) for j in (i, i + 1)]
        for blk in cb:
            blk.zero_grad()
        xc = xin.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            oc = cb[1](cb[0](xc)).float()
        oc.backward(dyt)
        checks = [(f"blocks {i},{i + 1} dx", xn.grad.float().permute(0, 3, 1, 2), xc.grad, xt.grad)]
        for k, j in enumerate((i, i + 1)):
            for (n, p), (_, q), (_, c) in zip(nb[j].named_parameters(), cb[k].named_parameters(),
                                              rb[j].named_parameters()):
                checks.append((f"block {j} {n}", p.grad, q.grad, c.grad))
        for n, a, c, t in checks:
            rn, cn = score(a, t)
            rc, cc = score(c, t)
            worst = max(worst, (rn - rc, f"{n}: {rn:.4f} vs autocast {rc:.4f}"))
            if not (rn <= 1.2 * rc + 0.01 and cn >= cc - 0.005):
                failures.append((n, round(rn, 4), round(rc, 4), round(cn, 5), round(cc, 5)))
        with torch.no_grad():
            r = rb[i + 1](rb[i](xin))
    print(f"{name}: largest native-minus-autocast error {worst[1]}")
    assert not failures, failures[:10]


def test_trajectory_tracks_fp32(gpu):
    """50 SGD steps of SimCLR on augmented class-structured synthetic images (the real
    GPU augmentation; all paths get the same views): native bf16 vs fp32 torch, with
    torch bf16 autocast as the control. Single steps of this trajectory are chaotic for
    ANY bf16 path (measured per-step gaps to fp32 up to 3 % native and 1.6 % autocast at
    lr 0.05, batch 128: tools/trajectory_probe.py), so the comparison is on 10-step window
    means: native within max(2.5 %, 2x the autocast gap, 2x the fp32 reference's own
    run-to-run gap) of fp32 in every window, and the fp32 and native losses must both fall by
    3 % (no collapsed run passes). The fp32 torch path is not deterministic on ROCm (MIOpen):
    its window-1 mean moved 35.7 -> 36.7 across five runs of the same native trajectory
    (round 4), so a second fp32 replica from the same init runs alongside and its gap to the
    first is part of the bar."""
    from simclr_pytorch_distributed_amd.data.augment import AugConfig, gpu_augment, nhwc8_to_nchw
    from simclr_pytorch_distributed_amd.data.datasets import build_dataset
    from simclr_pytorch_distributed_amd.losses.supcon import DistributedContrastiveLoss
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams, FusedSGD
    nat_m, ref_m = _models(gpu, "resnet18")
    ctl_m = _autocast_copy(gpu, ref_m)
    ref2_m = _models(gpu, "resnet18")[1]                  # same init (seed 0) as ref_m
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    lr0, B = 0.05, 128
    opt_n = FusedSGD(flat, lr=lr0, momentum=0.9, weight_decay=1e-4)
    opts = [torch.optim.SGD(m.parameters(), lr=lr0, momentum=0.9, weight_decay=1e-4) for m in (ref_m, ctl_m, ref2_m)]
    crit_n = DistributedContrastiveLoss("SimCLR", 0.5, backend="native")
    crit_t = DistributedContrastiveLoss("SimCLR", 0.5, backend="torch")
    ds = build_dataset("cifar10", None, True, True, 4096, 32, 0)
    data = torch.from_numpy(ds.images).to(gpu)
    aug = AugConfig.simclr(32, (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))
    L = {"n": [], "t": [], "c": [], "t2": []}
    for step in range(50):
        lr = lr0 * min(1.0, (step + 1) / 10)
        for o in opts:
            for gparam in o.param_groups:
                gparam["lr"] = lr
        opt_n.param_groups[0]["lr"] = lr          # step() syncs it to the device lr
        idx = torch.arange(B * step, B * step + B, device=gpu) % data.shape[0]
        v = gpu_augment(data, idx, aug, 1000 + step)          # [2B, 32, 32, 8] bf16
        vt = nhwc8_to_nchw(v)
        opt_n.zero_grad()
        ln = crit_n(runner.forward(v))
        ln.backward()
        opt_n.step()
        opts[0].zero_grad()
        lt = crit_t(ref_m(vt))
        lt.backward()
        opts[0].step()
        opts[1].zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lc = crit_t(ctl_m(vt).float())
        lc.backward()
        opts[1].step()
        opts[2].zero_grad()
        lt2 = crit_t(ref2_m(vt))
        lt2.backward()
        opts[2].step()
        for k, l in (("n", ln), ("t", lt), ("c", lc), ("t2", lt2)):
            L[k].append(float(l.detach()))
    torch.cuda.synchronize()
    W = {k: [sum(v[w:w + 10]) / 10 for w in range(0, 50, 10)] for k, v in L.items()}
    print("window means native", [round(v, 3) for v in W["n"]], "fp32", [round(v, 3) for v in W["t"]],
          "autocast", [round(v, 3) for v in W["c"]], "fp32 replica", [round(v, 3) for v in W["t2"]])
    mn, mt, mc, mt2 = W["n"], W["t"], W["c"], W["t2"]
    assert mt[0] - min(mt[-2:]) > 0.03 * mt[0], ("fp32 trajectory did not fall", mt)
    assert mn[0] - min(mn[-2:]) > 0.03 * mn[0], ("native trajectory did not fall", mn)
    for w in range(5):
        tol = max(0.025 * mt[w], 2 * abs(mc[w] - mt[w]), 2 * abs(mt2[w] - mt[w]))
        assert abs(mn[w] - mt[w]) <= tol, (w, mn[w], mt[w], mc[w], mt2[w])


def test_bn3_fold_forward_matches(gpu, monkeypatch):
    """Forward half of the BN3 fold (block_fwd fold_fwd: conv3 twice, BN3 + residual + ReLU in
    its epilogue, y3 never stored; backward Σdz·y3 from W3 and dzᵀ·a2) vs the backward-only
    fold on bottleneck pairs of ResNet-50 layers 1-2, the projection blocks l1.0 (stride 1) and
    l2.0 (stride 2, shortcut BN applied in conv3's epilogue) included: the block outputs, their ReLU
    bits and the BN running statistics are bit-identical (same conv, same statistics, the
    apply's operations in the same order); every gradient agrees to bf16 noise (Σdz·y3 from
    the unrounded y3)."""
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.ops import block as fb
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    monkeypatch.setattr(fb, "BN3_FOLD_ROWS_PER_K2", 0.0)
    monkeypatch.setattr(fb, "BN3_FOLD", True)
    nat_m, _ = _models(gpu, "resnet50")
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    wc = runner.weight_cache()
    nb = list(nat_m.encoder.blocks())
    g = torch.Generator().manual_seed(9)
    for i in (0, 1, 3, 4, 5):
        hw = 32 if i < 4 else 16
        x = torch.randn(16, hw, hw, nb[i].conv1.in_channels, generator=g).relu().to(gpu).to(torch.bfloat16)
        dy, res = None, {}
        bufs = [t for j in (i, i + 1) for t in nb[j].buffers()]
        snap = [t.clone() for t in bufs]
        for ff in (False, True):
            monkeypatch.setattr(fb, "FOLD_FWD", ff)
            with torch.no_grad():   # both runs update the running statistics from the same state
                for t, v in zip(bufs, snap):
                    t.copy_(v)
            flat.zero_grad()
            wc.refresh()
            chain = fb.BlockChain()
            xn = x.clone().requires_grad_(True)
            mid = fb.bottleneck(xn, nb[i], wc, True, None, chain, next_native=True)
            out = fb.bottleneck(mid, nb[i + 1], wc, True, None, chain)
            if dy is None:
                dy = torch.randn(out.shape, generator=g).to(gpu).to(torch.bfloat16)
            out.backward(dy)
            torch.cuda.synchronize()
            stats = [t.clone() for j in (i, i + 1) for t in nb[j].buffers()]
            res[ff] = (mid.detach().clone(), out.detach().clone(), stats,
                       [xn.grad.float().clone()] + [p.grad.float().clone() for j in (i, i + 1)
                                                    for p in nb[j].parameters()])
        assert torch.equal(res[True][0], res[False][0]) and torch.equal(res[True][1], res[False][1]), i
        for a, b in zip(res[True][2], res[False][2]):
            assert torch.equal(a, b), i
        names = ["dx"] + [f"block {j} {n}" for j in (i, i + 1) for n, _ in nb[j].named_parameters()]
        worst = max((float((a - b).norm() / (b.norm() + 1e-30)), n) for n, a, b in zip(names, res[True][3], res[False][3]))
        print(f"block {i}: worst fold_fwd vs fold gradient rel {worst[0]:.3g} ({worst[1]})")
        assert worst[0] < 2e-2, worst


def test_bn3_fold_matches_unfolded(gpu, monkeypatch):
    """BN3 fold (csrc/kernels/bnfold.hip) vs the materialised dy3 path on the same two-block
    chains (folding bottleneck -> next block) of ResNet-50 layers 1-2: every parameter
    gradient and the input gradient agree to bf16 rounding noise (masks are fixed by the
    forward, so only rounding points differ): rel <= 2e-2, cos >= 0.9998."""
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.ops import block as fb
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    monkeypatch.setattr(fb, "BN3_FOLD_ROWS_PER_K2", 0.0)   # fold at this small batch too
    nat_m, ref_m = _models(gpu, "resnet50")
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    wc = runner.weight_cache()
    nb = list(nat_m.encoder.blocks())
    g = torch.Generator().manual_seed(5)
    bad, seen = [], 0
    # l1.0 (projection, stride-1 shortcut: both BNs folded); l2.0 (strided projection: BN3
    # folded, dys from the masked dz); l1.1, l1.2, l2.1-l2.3, l3.1 (identity; K = 64, 128, 256)
    for i in (0, 1, 2, 3, 4, 5, 6, 8):
        c_in = nb[i].conv1.in_channels
        hw = 32 if i < 4 else (16 if i < 7 else 8)   # block inputs (l2.0 reads 32x32)
        x = torch.randn(16, hw, hw, c_in, generator=g).relu().to(gpu).to(torch.bfloat16)
        dy = None
        res = {}
        for fold in (False, True):
            monkeypatch.setattr(fb, "BN3_FOLD", fold)
            flat.zero_grad()
            wc.refresh()
            chain = fb.BlockChain()
            xn = x.clone().requires_grad_(True)
            out = fb.bottleneck(fb.bottleneck(xn, nb[i], wc, True, None, chain, next_native=True), nb[i + 1], wc, True,
                                None, chain)
            if dy is None:
                dy = torch.randn(out.shape, generator=g).to(gpu).to(torch.bfloat16)
            out.backward(dy)
            torch.cuda.synchronize()
            res[fold] = [xn.grad.float().clone()] + [p.grad.float().clone() for j in (i, i + 1)
                                                     for p in nb[j].parameters()]
        names = ["dx"] + [f"block {j} {n}" for j in (i, i + 1) for n, _ in nb[j].named_parameters()]
        for n, a, b in zip(names, res[True], res[False]):
            a, b = a.double().flatten(), b.double().flatten()
            rel = float((a - b).norm() / (b.norm() + 1e-30))
            cos = float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))
            seen += 1
            if not (rel <= 2e-2 and cos >= 0.9998):
                bad.append((f"pair {i}: {n}", round(rel, 5), round(cos, 6)))
    assert seen > 0
    assert not bad, bad[:10]


def test_bn3_fold_full_batch_gradients(gpu, monkeypatch):
    """The BN3 fold at the headline batch (512 views of 32x32, where its Grams and column
    sums run over 524288 rows in layer 1): whole-network parameter gradients, fold vs the
    materialised dy3 path, same weights / input / forward (masks identical) — every one of
    the 161 parameters within bf16 rounding noise (rel <= 5e-2, cos >= 0.999; measured worst
    layer1.2.bn2.bias 0.033 / 0.99945). Regression test for the swamped-addend drift (0.2 rel
    when the fold's addend was added after the bf16 rounding)."""
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner, to_nhwc_input
    from simclr_pytorch_distributed_amd.ops import block as fb
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    nat_m, _ = _models(gpu, "resnet50")
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    x = to_nhwc_input(_images(gpu, 512, seed=4))
    G = torch.randn(512, 128, generator=torch.Generator().manual_seed(6)).to(gpu)
    grads = {}
    for fold in (False, True):
        monkeypatch.setattr(fb, "BN3_FOLD", fold)
        flat.zero_grad()
        (runner.forward(x) * G).sum().backward()
        torch.cuda.synchronize()
        grads[fold] = [p.grad.double().flatten().clone() for p in nat_m.parameters()]
    bad, worst = [], (0.0, "")
    for (n, _), a, b in zip(nat_m.named_parameters(), grads[True], grads[False]):
        rel = float((a - b).norm() / (b.norm() + 1e-30))
        cos = float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))
        worst = max(worst, (rel, f"{n}: rel {rel:.4g} cos {cos:.6f}"))
        if not (rel <= 5e-2 and cos >= 0.999):
            bad.append((n, round(rel, 5), round(cos, 6)))
    print(f"fold vs unfolded at 512 views, worst: {worst[1]}")
    assert not bad, bad[:10]


@pytest.mark.parametrize("fold", [False, True])
def test_stage_gradients_match_fp32(gpu, fold, monkeypatch):
    """ResNet-50 encoder gradient gate at STAGE granularity: each of layer1-4 is
    teacher-forced as a unit — input = the fp32 network's activation into that stage
    (bf16-rounded), a random bf16 upstream gradient at its output — and run through the
    native executor (every block of the stage chained: cross-block BN-statistic hand-off,
    BN3 / shortcut folds, compact strided-shortcut gradients, ReLU bitmasks), fp32 torch
    and torch bf16 autocast. Every parameter gradient of the stage and its input gradient
    must stay inside the autocast envelope. Two bars: per stage, the MEDIAN over tensors of
    native rel / autocast rel <= 1.2 (a systematic bias moves every tensor), and per tensor
    rel <= 1.5x autocast + 0.02 and cos >= autocast cos - 0.02 (outliers: with ~40 tensors a
    stage, two independent bf16 implementations differ by more than 1.2x on a few of them —
    layer1.0.bn1.weight 0.186 vs 0.141 on one box, within 1.2x on another). fold=True forces
    the BN3 fold wherever K <= 128."""
    import copy
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.ops import block as fb
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    monkeypatch.setattr(fb, "BN3_FOLD", fold)
    if fold:
        monkeypatch.setattr(fb, "BN3_FOLD_ROWS_PER_K2", 0.0)
        monkeypatch.setattr(fb, "BN3_FOLD_MAXK", 128)
    nat_m, ref_m = _models(gpu, "resnet50")
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    wc = runner.weight_cache()
    g = torch.Generator().manual_seed(11)
    enc_n, enc_r = nat_m.encoder, ref_m.encoder
    with torch.no_grad():
        r = torch.relu(enc_r.bn1(enc_r.conv1(_images(gpu, 32))))

    def score(a, b):
        a, b = a.double().flatten(), b.double().flatten()
        return float((a - b).norm() / (b.norm() + 1e-30)), float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))

    failures, report = [], []
    for stage in ("layer1", "layer2", "layer3", "layer4"):
        sn, sr = getattr(enc_n, stage), getattr(enc_r, stage)
        xin = r.to(torch.bfloat16).float().detach()
        flat.zero_grad()
        wc.refresh()
        chain = fb.BlockChain()
        xn = xin.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).requires_grad_(True)
        out = xn
        for j, blk in enumerate(sn):
            out = fb.bottleneck(out, blk, wc, True, None, chain, next_native=j + 1 < len(sn))
        dy = torch.randn(out.shape, generator=g).to(gpu).to(torch.bfloat16)
        out.backward(dy)
        torch.cuda.synchronize()
        dyt = dy.float().permute(0, 3, 1, 2)
        xt = xin.clone().requires_grad_(True)
        sr.zero_grad()
        sr(xt).backward(dyt)
        sc = copy.deepcopy(sr).to(memory_format=torch.channels_last)
        sc.zero_grad()
        xc = xin.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            oc = sc(xc).float()
        oc.backward(dyt)
        checks = [(f"{stage} dx", xn.grad.float().permute(0, 3, 1, 2), xc.grad, xt.grad)]
        for (n, p), (_, q), (_, c) in zip(sn.named_parameters(), sc.named_parameters(), sr.named_parameters()):
            checks.append((f"{stage}.{n}", p.grad, q.grad, c.grad))
        worst = (-1.0, "")
        ratios = []
        for n, a, c, t in checks:
            rn, cn = score(a, t)
            rc, cc = score(c, t)
            ratios.append(rn / max(rc, 1e-12))
            worst = max(worst, (rn - rc, f"{n}: {rn:.4f} vs autocast {rc:.4f}"))
            if not (rn <= 1.5 * rc + 0.02 and cn >= cc - 0.02):
                failures.append((n, round(rn, 4), round(rc, 4), round(cn, 5), round(cc, 5)))
        med = sorted(ratios)[len(ratios) // 2]
        if med > 1.2:
            failures.append((stage, "median native/autocast rel", round(med, 4)))
        report.append(f"{stage} ({len(checks)} tensors) median native/autocast rel {med:.3f}, "
                      f"worst native-minus-autocast {worst[1]}")
        with torch.no_grad():
            r = sr(xin)
    print("\n".join(report))
    assert not failures, failures[:10]


def test_teacher_forced_trajectory_gradients(gpu):
    """ResNet-50 along an fp32 SimCLR trajectory (12 SGD steps, lr 0.05 with the 10-step
    ramp, 64 images x 2 views of the class-structured synthetic set through the GPU
    augmentation): before every step the fp32 weights are copied into the native model and
    into a torch bf16-autocast control, and the whole-network gradients of the SAME loss on
    the SAME views are compared (tools/trajectory_tf.py). At this network's random init ANY
    bf16 path's gradient is ~100 % off fp32 (ReLU-mask flips compound over 16 blocks:
    measured global rel 1.2-1.3 for native and autocast alike, profiles/
    trajectory_probe_r50_r3.txt), so the gate is relative: the native error, averaged over
    the steps, within 1.2x the autocast error + 0.02, and every step's native loss within
    2e-3 (relative) of fp32. A systematic native gradient bias fails the first bar; the
    free-running trajectories themselves are chaotic (two fp32 replicas separate too)."""
    from simclr_pytorch_distributed_amd.data.augment import AugConfig, gpu_augment, nhwc8_to_nchw
    from simclr_pytorch_distributed_amd.data.datasets import build_dataset
    from simclr_pytorch_distributed_amd.losses.supcon import DistributedContrastiveLoss
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    nat_m, ref_m = _models(gpu, "resnet50")
    ctl_m = _autocast_copy(gpu, ref_m)
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    opt = torch.optim.SGD(ref_m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    crit_n = DistributedContrastiveLoss("SimCLR", 0.5, backend="native")
    crit_t = DistributedContrastiveLoss("SimCLR", 0.5, backend="torch")
    ds = build_dataset("cifar10", None, True, True, 2048, 32, 0)
    data = torch.from_numpy(ds.images).to(gpu)
    aug = AugConfig.simclr(32, (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010))
    B, errs, rows = 64, {"n": [], "c": []}, []
    for step in range(12):
        for gp in opt.param_groups:
            gp["lr"] = 0.05 * min(1.0, (step + 1) / 10)
        with torch.no_grad():
            sd = ref_m.state_dict()
            nat_m.load_state_dict(sd)
            ctl_m.load_state_dict(sd)
        idx = torch.arange(B * step, B * step + B, device=gpu) % data.shape[0]
        v = gpu_augment(data, idx, aug, 2000 + step)
        vt = nhwc8_to_nchw(v)
        flat.zero_grad()
        ln = crit_n(runner.forward(v))
        ln.backward()
        opt.zero_grad()
        lt = crit_t(ref_m(vt))
        lt.backward()
        ctl_m.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lc = crit_t(ctl_m(vt).float())
        lc.backward()
        torch.cuda.synchronize()
        gt = torch.cat([p.grad.double().flatten() for p in ref_m.parameters()])
        for k, mdl in (("n", nat_m), ("c", ctl_m)):
            gg = torch.cat([p.grad.double().flatten() for p in mdl.parameters()])
            errs[k].append(float((gg - gt).norm() / gt.norm()))
        rows.append((float(lt.detach()), float(ln.detach()), float(lc.detach())))
        opt.step()
    mn, mc = sum(errs["n"]) / len(errs["n"]), sum(errs["c"]) / len(errs["c"])
    print(f"mean whole-network gradient rel error vs fp32: native {mn:.4f}, autocast {mc:.4f}; per step native "
          f"{[round(e, 3) for e in errs['n']]} autocast {[round(e, 3) for e in errs['c']]}")
    assert mn <= 1.2 * mc + 0.02, (mn, mc)
    for lt_, ln_, _ in rows:
        assert abs(ln_ - lt_) <= 2e-3 * abs(lt_), rows


def test_merged_splitk_reductions_bit_identical(gpu):
    """The side-stream split-K reductions of a residual block merged into ONE multi-tensor
    launch (splitk_merge_set, the default) give every parameter gradient bit for bit as one
    reduction launch per weight gradient: same per-element summation order. A repeat of the
    unmerged step first pins that the step itself is deterministic (the control)."""
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner, to_nhwc_input
    from simclr_pytorch_distributed_amd.ops import _ext
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    m = _ext.require()
    nat_m, _ = _models(gpu, "resnet50")
    flat = FlatParams(nat_m)
    runner = ModelRunner(nat_m, "native", master=flat.flat)
    x = to_nhwc_input(_images(gpu, 128, seed=4))
    G = torch.randn(128, 128, generator=torch.Generator().manual_seed(6)).to(gpu)
    grads = []
    prev = m.splitk_merge_set(False)
    try:
        for merge in (False, False, True):
            m.splitk_merge_set(merge)
            flat.zero_grad()
            (runner.forward(x) * G).sum().backward()
            torch.cuda.synchronize()
            grads.append(flat.grad.detach().clone())
    finally:
        m.splitk_merge_set(bool(prev))
    assert torch.equal(grads[0], grads[1]), "unmerged step is not deterministic"
    assert torch.equal(grads[0], grads[2])
