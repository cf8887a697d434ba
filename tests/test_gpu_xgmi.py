"""One-shot xGMI all-reduce protocol, emulated with W virtual ranks (W blocks of one launch)
on the single test GPU: slot/flag/parity logic over several calls (both arena parities,
reuse), bit-identical results on every rank, equal to the rank-ordered fp64 sum."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("n", [1, 130, 4096])
def test_oneshot_emulation(gpu, world, n):
    from simclr_pytorch_distributed_amd.parallel.xgmi import emulate
    torch.manual_seed(world * 1000 + n)
    x = torch.randn(world, n, dtype=torch.float64, device=gpu)
    out = emulate(x, iters=5)
    ref = x[0].clone()
    for q in range(1, world):
        ref = ref + x[q]
    for r in range(world):
        assert torch.equal(out[r], out[0])
    assert torch.allclose(out[0], ref, rtol=0, atol=1e-12)


def test_small_allreduce_routing(gpu):
    """comm.small_all_reduce_ dispatches to a registered implementation for fp64 GPU tensors."""
    from simclr_pytorch_distributed_amd.parallel import comm

    class Fake:
        calls = 0

        def all_reduce_(self, x):
            Fake.calls += 1
            return x.mul_(2)

    comm.set_small_allreduce(None, Fake())
    try:
        import torch.distributed as dist
        x = torch.ones(4, dtype=torch.float64, device=gpu)
        comm.small_all_reduce_(x, dist.group.WORLD if dist.is_initialized() else None)
        assert Fake.calls == 1 and torch.equal(x, torch.full_like(x, 2.0))
    finally:
        comm.set_small_allreduce(None, None)


@pytest.mark.parametrize("world", [2, 8])
def test_fused_exchange_emulated(gpu, world):
    """Fused SyncBN exchange (csrc/kernels/bn.hip col_reduce + XgmiCol), W emulated ranks on
    this GPU, each with its OWN slab: the returned sums are the global (all-rank) column
    sums. A sequence of calls with varying channel counts exercises both arena parities,
    per-group flags of groups that a call skips, and 1..3 statistic sets."""
    m = __import__("simclr_pytorch_distributed_amd.ops._ext", fromlist=["require"]).require()
    h = m.xgmi_emu_small_comm(world)
    try:
        g = torch.Generator(device="cpu").manual_seed(world)
        for it, (rows, ns, C) in enumerate([(64, 2, 64), (513, 3, 2048), (1, 2, 256), (96, 2, 2048),
                                            (7, 1, 130), (300, 3, 512), (64, 2, 64), (33, 2, 1000)]):
            slab = torch.randn(world, rows, ns, C, generator=g).to(gpu)
            got = m.syncbn_exchange_sums(h, slab)
            exp = slab.double().sum(dim=(0, 1))
            torch.cuda.synchronize()
            assert got.shape == (ns, C)
            assert torch.allclose(got, exp, rtol=1e-12, atol=1e-9), (it, float((got - exp).abs().max()))
        assert m.small_comm_kind(h) == 4
    finally:
        m.small_comm_destroy(h)
