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
