"""CIFAR-stem ResNet-18/34/50/101 encoders, projection heads and classifiers.

Module tree, parameter names and initialisation follow the reference
(networks/resnet_big.py:7-204) so that checkpoints cross-load in both directions:
``encoder.conv1``, ``encoder.bn1``, ``encoder.layer{1..4}.{i}.{conv,bn}{1,2,3}``,
``encoder.layer{k}.0.shortcut.{0,1}`` and ``head.{0,2}`` (MLP) / ``head`` (linear).

What is different (MI355X-first):

* The modules only *own* parameters and buffers. How a forward pass executes is
  chosen per call by :mod:`simclr_pytorch_distributed_amd.models.executor`:
  ``torch`` (stock ops — CPU runs and the numerics oracle) or ``native`` (NHWC bf16
  hand-written gfx950 kernels: implicit-GEMM MFMA convolutions with fused BatchNorm
  statistics, fused BN-apply/residual/ReLU, see ``ops/``).
* ``stem='imagenet'`` adds the 7x7/2 + maxpool stem for 224² inputs (SURVEY.md §7.4
  item 4); the default ``'cifar'`` stem is the reference's 3x3/1 conv with no maxpool
  (networks/resnet_big.py:75-77).
* ``zero_init_residual`` and the ``is_last``/``preact`` outputs are kept for API
  parity (networks/resnet_big.py:31-34, 64-67, 94-99).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "BasicBlock", "Bottleneck", "ResNet", "resnet18", "resnet34", "resnet50", "resnet101",
    "model_dict", "LinearBatchNorm", "SupConResNet", "SupCEResNet", "LinearClassifier",
]


class BasicBlock(nn.Module):
    """Two 3x3 convs (reference networks/resnet_big.py:7-35)."""

    expansion = 1

    def __init__(self, in_planes: int, planes: int, stride: int = 1, is_last: bool = False):
        super().__init__()
        self.is_last = is_last
        self.stride = stride
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, 1, stride, bias=False),
                nn.BatchNorm2d(self.expansion * planes),
            )

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out = out + self.shortcut(x)
        preact = out
        out = F.relu(out)
        return (out, preact) if self.is_last else out


class Bottleneck(nn.Module):
    """1x1 -> 3x3(stride) -> 1x1 bottleneck, ResNet v1.5 (networks/resnet_big.py:38-67)."""

    expansion = 4

    def __init__(self, in_planes: int, planes: int, stride: int = 1, is_last: bool = False):
        super().__init__()
        self.is_last = is_last
        self.stride = stride
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, self.expansion * planes, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(self.expansion * planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, 1, stride, bias=False),
                nn.BatchNorm2d(self.expansion * planes),
            )

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        out = out + self.shortcut(x)
        preact = out
        out = F.relu(out)
        return (out, preact) if self.is_last else out


class ResNet(nn.Module):
    """ResNet trunk with a CIFAR (3x3/1, no maxpool) or ImageNet (7x7/2 + maxpool) stem.

    Reference: networks/resnet_big.py:70-118. ``layer`` (dead argument of the
    reference forward) is accepted and ignored.
    """

    def __init__(self, block, num_blocks, in_channel: int = 3, zero_init_residual: bool = False,
                 stem: str = "cifar"):
        super().__init__()
        self.in_planes = 64
        self.block = block
        self.stem = stem
        if stem == "cifar":
            self.conv1 = nn.Conv2d(in_channel, 64, 3, 1, 1, bias=False)
        elif stem == "imagenet":
            self.conv1 = nn.Conv2d(in_channel, 64, 7, 2, 3, bias=False)
        else:
            raise ValueError(f"unknown stem: {stem}")
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], 1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], 2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], 2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, num_blocks, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    def blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            yield from layer

    def forward(self, x, layer: int = 100):
        out = F.relu(self.bn1(self.conv1(x)))
        if self.stem == "imagenet":
            out = F.max_pool2d(out, 3, 2, 1)
        out = self.layer1(out)
        out = self.layer2(out)
        out = self.layer3(out)
        out = self.layer4(out)
        out = self.avgpool(out)
        return torch.flatten(out, 1)


def resnet18(**kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], **kw)


def resnet34(**kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], **kw)


def resnet50(**kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], **kw)


def resnet101(**kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], **kw)


# name -> (constructor, encoder output dim)   (networks/resnet_big.py:137-142)
model_dict = {
    "resnet18": [resnet18, 512],
    "resnet34": [resnet34, 512],
    "resnet50": [resnet50, 2048],
    "resnet101": [resnet101, 2048],
}


class LinearBatchNorm(nn.Module):
    """BatchNorm1d expressed as BatchNorm2d (networks/resnet_big.py:145-156)."""

    def __init__(self, dim: int, affine: bool = True):
        super().__init__()
        self.dim = dim
        self.bn = nn.BatchNorm2d(dim, affine=affine)

    def forward(self, x):
        return self.bn(x.view(-1, self.dim, 1, 1)).view(-1, self.dim)


class SupConResNet(nn.Module):
    """Encoder + projection head (networks/resnet_big.py:159-181).

    ``forward`` returns the *un-normalised* projection, as the reference does; the
    L2-normalisation is fused into the contrastive-loss kernel.
    """

    def __init__(self, name: str = "resnet50", head: str = "mlp", feat_dim: int = 128,
                 stem: str = "cifar", zero_init_residual: bool = False):
        super().__init__()
        model_fun, dim_in = model_dict[name]
        self.name = name
        self.dim_in = dim_in
        self.feat_dim = feat_dim
        self.head_type = head
        self.encoder = model_fun(stem=stem, zero_init_residual=zero_init_residual)
        if head == "linear":
            self.head = nn.Linear(dim_in, feat_dim)
        elif head == "mlp":
            self.head = nn.Sequential(nn.Linear(dim_in, dim_in), nn.ReLU(inplace=True),
                                      nn.Linear(dim_in, feat_dim))
        else:
            raise NotImplementedError(f"head not supported: {head}")

    def forward(self, x):
        return self.head(self.encoder(x))


class SupCEResNet(nn.Module):
    """Encoder + linear classifier for supervised CE (networks/resnet_big.py:184-193)."""

    def __init__(self, name: str = "resnet50", num_classes: int = 10, stem: str = "cifar"):
        super().__init__()
        model_fun, dim_in = model_dict[name]
        self.encoder = model_fun(stem=stem)
        self.fc = nn.Linear(dim_in, num_classes)

    def forward(self, x):
        return self.fc(self.encoder(x))


class LinearClassifier(nn.Module):
    """Linear probe on frozen encoder features (networks/resnet_big.py:196-204)."""

    def __init__(self, name: str = "resnet50", num_classes: int = 10):
        super().__init__()
        _, feat_dim = model_dict[name]
        self.fc = nn.Linear(feat_dim, num_classes)

    def forward(self, features):
        return self.fc(features)
