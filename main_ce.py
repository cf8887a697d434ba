"""Supervised data loaders (reference main_ce.py:19-68 keeps only ``set_loader``).

``set_loader(opt)`` returns (train, val) in-memory datasets plus the GPU augmentation
configs used by the linear probe: RandomResizedCrop(32, scale=(0.2,1)) + flip +
normalize for training, normalize only for validation.
"""
from simclr_pytorch_distributed_amd.config import DATASET_STATS
from simclr_pytorch_distributed_amd.data.augment import AugConfig
from simclr_pytorch_distributed_amd.data.datasets import build_dataset


def set_loader(opt):
    if opt.dataset not in DATASET_STATS:
        raise ValueError("dataset not supported: {}".format(opt.dataset))
    mean, std = DATASET_STATS[opt.dataset]
    synthetic = getattr(opt, "synthetic", False)
    train = build_dataset(opt.dataset, opt.data_folder, True, synthetic)
    val = build_dataset(opt.dataset, opt.data_folder, False, synthetic)
    return (train, AugConfig.linear_train(32, mean, std)), (val, AugConfig.evaluation(32, mean, std))
