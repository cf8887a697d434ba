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


def test_synthetic_train_val_share_class_statistics():
    """Train and validation splits of the synthetic dataset use the same per-class image
    statistics (else a linear probe cannot transfer), with different samples."""
    import numpy as np
    from simclr_pytorch_distributed_amd.data.datasets import build_dataset
    tr = build_dataset("cifar10", None, True, True, 2000, 32, 3)
    va = build_dataset("cifar10", None, False, True, 2000, 32, 3)
    assert not np.array_equal(tr.images[:10], va.images[:10])
    for c in range(10):
        mt = tr.images[tr.labels == c].reshape(-1, 3).mean(0)
        mv = va.images[va.labels == c].reshape(-1, 3).mean(0)
        assert np.abs(mt - mv).max() < 6.0, (c, mt, mv)
