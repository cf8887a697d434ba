"""BN3 fold eligibility (simclr_pytorch_distributed_amd/ops/block.py, csrc/kernels/bnfold.hip):
which bottlenecks fold for the ResNet-50 shapes of the BASELINE configs. CPU only."""
import torch

from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
from simclr_pytorch_distributed_amd.ops import block as fb


def _plan(monkeypatch, views, size, stem):
    monkeypatch.setattr(fb, "BN3_FOLD", True)
    monkeypatch.setattr(fb, "BN3_FOLD_MAXK", 512)
    monkeypatch.setattr(fb, "BN3_FOLD_ROWS_PER_K2", 2.0)
    m = SupConResNet("resnet50")
    hw = size // 4 if stem == "imagenet" else size
    plan = []
    for layer, stride in ((m.encoder.layer1, 1), (m.encoder.layer2, 2), (m.encoder.layer3, 2), (m.encoder.layer4, 2)):
        for j, blk in enumerate(layer):
            if j == 0:
                hw //= stride
            (convs, bns, bottle, proj), _ = fb._block_info(blk)
            rows = views * hw * hw
            f = fb._fold_eligible(convs, bottle, proj, rows)
            plan.append((f, bool(f and proj and fb._fold_shortcut(convs, rows))))
    return plan


def test_cifar_headline_folds_layers_1_2(monkeypatch):
    plan = _plan(monkeypatch, 512, 32, "cifar")
    assert [f for f, _ in plan] == [True] * 7 + [False] * 9     # layers 1-2 (3 + 4 blocks)
    assert [s for _, s in plan] == [True] + [False] * 15        # only l1.0 has a stride-1 shortcut


def test_imagenet_224_folds_layers_1_3(monkeypatch):
    plan = _plan(monkeypatch, 1024, 224, "imagenet")
    assert [f for f, _ in plan] == [True] * 13 + [False] * 3     # layers 1-3


def test_fold_off_and_basic_blocks(monkeypatch):
    monkeypatch.setattr(fb, "BN3_FOLD", False)
    m = SupConResNet("resnet50")
    (convs, bns, bottle, proj), _ = fb._block_info(m.encoder.layer1[1])
    assert not fb._fold_eligible(convs, bottle, proj, 1 << 30)
    monkeypatch.setattr(fb, "BN3_FOLD", True)
    r18 = SupConResNet("resnet18")
    (convs, bns, bottle, proj), _ = fb._block_info(r18.encoder.layer1[0])
    assert not fb._fold_eligible(convs, bottle, proj, 1 << 30)   # basic blocks have no conv3
    assert torch.is_tensor(fb._fold_marker(torch.zeros(1)))
