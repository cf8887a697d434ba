"""Native small communicators (csrc/bindings/comm_ops.cpp) and the SyncBN path of the C++
block executor (csrc/bindings/conv_bn_ops.cpp block_fwd / block_bwd with a comm handle).

The box has one GPU, so multi-rank RCCL cannot run here: the RCCL kind is exercised
with a 1-rank communicator (linking against torch's librccl, ncclCommInitRank,
ncclAllReduce on the compute stream), and the executor's cross-rank code path
(reduce -> all-reduce -> finalize / coefficients) with the EMU kind: W virtual ranks that
hold identical data, whose sum is x·W. SyncBN over W identical replicas must give the
single-process statistics (so identical outputs, dx and conv weight gradients) and the
single-process dγ/dβ: each rank writes 1/W of the globally summed Σdz, Σdz·ŷ into its
gradient sinks (its share; the bucket reducer's mean then gives torch's global / W).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _m():
    from simclr_pytorch_distributed_amd.ops import _ext
    return _ext.require()


def test_rccl_single_rank_comm(gpu):
    m = _m()
    uid = m.rccl_unique_id()
    assert uid.dtype == torch.uint8 and uid.numel() == 128
    h = m.rccl_comm_init(uid, 1, 0)
    try:
        assert m.small_comm_world(h) == 1
        for dt in (torch.float64, torch.float32):
            x = torch.randn(1000, dtype=dt, device=gpu)
            y = x.clone()
            m.small_all_reduce_(h, y)
            torch.cuda.synchronize()
            assert torch.equal(x, y)
    finally:
        m.small_comm_destroy(h)


def test_emu_comm_sum(gpu):
    m = _m()
    h = m.emu_small_comm(4)
    x = torch.randn(64, dtype=torch.float64, device=gpu)
    y = x.clone()
    m.small_all_reduce_(h, y)
    assert torch.equal(y, 4 * x)
    m.small_comm_destroy(h)


@pytest.mark.parametrize("kind,W", [("emu", 2), ("xemu", 2), ("xemu", 8)])
@pytest.mark.parametrize("which", ["layer1.0", "layer1.1", "layer2.0", "layer3.0"])
@pytest.mark.parametrize("name", ["resnet50", "resnet18"])
def test_native_executor_syncbn_path(gpu, name, which, kind, W):
    """Two chained blocks through the executor's SyncBN path over W identical virtual ranks
    vs the single-process path: EVERY parameter gradient of both blocks (incl. the folded
    bn3 / conv3 / shortcut of ResNet-50 layer 1-2 blocks: 8 images x 32² = 8192 rows fold
    K = 64), the input gradient, outputs and running statistics. kind 'emu': reduce ->
    all-reduce (x·W) -> finalize; 'xemu': the fused exchange (reduce + exchange + epilogue
    in one launch, W z-slices of each launch talking through W device-memory arenas).
    With a power-of-two W the global statistics are exact multiples of the local ones."""
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    from simclr_pytorch_distributed_amd.ops import block
    from simclr_pytorch_distributed_amd.optim.flat import FlatParams
    m = _m()
    h = m.emu_small_comm(W) if kind == "emu" else m.xgmi_emu_small_comm(W)
    torch.manual_seed(0)
    models = [SupConResNet(name).to(gpu).to(memory_format=torch.channels_last) for _ in range(2)]
    models[1].load_state_dict(models[0].state_dict())
    lay, idx = which.split(".")
    if name == "resnet18" and which == "layer1.1":
        pytest.skip("resnet18 layer1 has two blocks: layer1.0 covers the pair")
    cin = getattr(models[0].encoder, lay)[int(idx)].conv1.in_channels
    hw = 32 if lay in ("layer1", "layer2") else 16
    x = torch.randn(8, hw, hw, cin, device=gpu).to(torch.bfloat16)
    dout = None
    res = []
    for mdl, hh in zip(models, (0, h)):
        flat = FlatParams(mdl)
        runner = ModelRunner(mdl, "native", master=flat.flat, fused=True)
        wc = runner.weight_cache()
        wc.refresh()
        blk = getattr(mdl.encoder, lay)[int(idx)]
        info, params = block._block_info(blk)
        flat.zero_grad()
        xi = x.clone().requires_grad_(True)
        # two chained blocks (the second's final dgrad hands the first its output-BN sums)
        nxt = getattr(mdl.encoder, lay)[int(idx) + 1]
        ninfo, nparams = block._block_info(nxt)
        link = block.BlockLink()
        # layer-1/2 identity bottlenecks also fold their BN3 forward (no y3; Σdz·y3 from W3, dzᵀa2)
        ff = block._fold_fwd(xi, info, True, True)
        mid = block._NativeBlock.apply(xi, blk, wc, True, info, hh, None, link, ff, *params)
        out = block._NativeBlock.apply(mid, nxt, wc, True, ninfo, hh, link, None, False, *nparams)
        if dout is None:
            dout = torch.randn_like(out)
        out.backward(dout)
        torch.cuda.synchronize()
        res.append((out.detach().float(), xi.grad.float(), blk, nxt))
    (o0, dx0, b0, n0), (o1, dx1, b1, n1) = res
    assert torch.equal(o0, o1)
    assert torch.allclose(dx0, dx1, rtol=1e-2, atol=1e-3)
    for a, b in ((b0, b1), (n0, n1)):
        for (na, ma), (_, mb) in zip(a.named_modules(), b.named_modules()):
            if isinstance(ma, torch.nn.BatchNorm2d):
                # running_var is updated with the UNBIASED variance: n/(n-1) over the global
                # row count, which differs between 1 and W ranks
                assert torch.equal(ma.running_mean, mb.running_mean), na
                assert torch.allclose(ma.running_var, mb.running_var, rtol=1e-3), na
    worst, bad, seen = (0.0, ""), [], 0
    for tag, a, b in (("blk", b0, b1), ("next", n0, n1)):
        for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            seen += 1
            g0, g1 = p.grad.double(), q.grad.double()
            rel = float((g1 - g0).norm() / (g0.norm() + 1e-30))
            worst = max(worst, (rel, f"{tag}.{n}"))
            if not torch.allclose(g0, g1, rtol=1e-3, atol=1e-5):
                bad.append((f"{tag}.{n}", rel))
    print(f"{name} {which} {kind} W={W}: {seen} parameters, worst rel {worst[0]:.3g} ({worst[1]})")
    assert seen >= (12 if name == "resnet18" else 18)
    assert not bad, bad
    m.small_comm_destroy(h)


@pytest.mark.parametrize("kind", ["rccl1", "emu3"])
def test_native_gather_scatter(gpu, kind):
    """Embedding exchange of the contrastive loss on a native communicator:
    rank-major all-gather, SUM reduce-scatter, and the fused normalise-into-C + in-place
    gather with its autograd backward, vs plain torch (1-rank RCCL: the real ncclAllGather /
    ncclReduceScatter calls; emulated W=3: identical virtual ranks)."""
    import torch.nn.functional as F
    from simclr_pytorch_distributed_amd.ops.contrastive import row_normalize_gather
    m = _m()
    h = m.rccl_comm_init(m.rccl_unique_id(), 1, 0) if kind == "rccl1" else m.emu_small_comm(3)
    W = m.small_comm_world(h)
    try:
        x = torch.randn(37, 128, device=gpu)
        g = m.small_all_gather(h, x)
        assert torch.equal(g, x.repeat(W, 1))
        lab = torch.randint(0, 10, (37,), device=gpu)
        assert torch.equal(m.small_all_gather(h, lab), lab.repeat(W))
        gc = torch.randn(W * 37, 128, device=gpu)
        assert torch.allclose(m.small_reduce_scatter(h, gc), W * gc[:37])
        xa = x.clone().requires_grad_(True)
        C = row_normalize_gather(xa, h)
        ref = F.normalize(x.double(), dim=1)
        assert torch.allclose(C.double(), ref.repeat(W, 1), rtol=1e-6, atol=1e-6)
        C.backward(gc)
        xr = x.double().clone().requires_grad_(True)
        F.normalize(xr, dim=1).backward(W * gc[:37].double())   # identical ranks: W x own block
        assert torch.allclose(xa.grad.double(), xr.grad, rtol=1e-4, atol=1e-5)
        assert m.small_comm_kind(h) == (1 if kind == "rccl1" else 3) and m.small_comm_rank(h) == 0
    finally:
        m.small_comm_destroy(h)
