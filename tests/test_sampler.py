import numpy as np

from simclr_pytorch_distributed_amd.data.sampler import DistributedIndexSampler


def test_iters_per_epoch_cifar_2gpu():
    s = DistributedIndexSampler(50000, 128, world=2, rank=0)
    assert len(s) == 195


def test_shards_disjoint_and_cover():
    ws = 3
    shards = [DistributedIndexSampler(100, 4, world=ws, rank=r, seed=5) for r in range(ws)]
    for s in shards:
        s.set_epoch(2)
    idx = np.concatenate([s.indices() for s in shards])
    assert len(idx) == 102 and set(idx.tolist()) == set(range(100))
    a = DistributedIndexSampler(100, 4, seed=5)
    a.set_epoch(1)
    b = DistributedIndexSampler(100, 4, seed=5)
    b.set_epoch(2)
    assert not np.array_equal(a.indices(), b.indices())
