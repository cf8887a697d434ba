"""Execution of the ResNet modules on the native gfx950 path.

The modules in ``models/resnet.py`` own parameters/buffers with the reference's names;
this executor walks them and issues the fused native ops instead of ``nn.Conv2d`` /
``nn.BatchNorm2d``:

* activations NHWC bf16, produced and consumed by the implicit-GEMM MFMA conv kernels;
* every conv (training) emits its BN statistics from the epilogue; every BN+ReLU (and
  BN+shortcut-BN+add+ReLU) is one fused elementwise pass; each residual block's forward
  and backward kernel sequence is issued by ONE C++ call (ops/block.py ->
  csrc/bindings/conv_bn_ops.cpp block_fwd / block_bwd); SyncBN statistics are exchanged
  by the native communicator inside that call (the fused xGMI exchange by default:
  reduce + exchange + finalize in one launch per BN);
* global average pooling is a native kernel (pool.hip) and the projection head one
  autograd node whose GEMMs run on the same MFMA kernels with bias/ReLU epilogues
  (ops/head.py); the per-op path below (``fused=False``) remains as a reference executor.

Reference forward: networks/resnet_big.py:57-67 (Bottleneck), 24-35 (BasicBlock),
110-118 (ResNet), 177-181 (SupConResNet).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..ops.bn import bn_act, bn_add_act
from ..ops.conv import conv2d_nhwc
from ..ops.pool import global_avgpool_nhwc, maxpool_nhwc
from .resnet import BasicBlock, Bottleneck, ResNet

INPUT_CHANNELS_PADDED = 8   # NHWC input images carry 3 channels padded to 8 (16-byte rows)


def _bottleneck(b: Bottleneck, x, training, group):
    st = training
    y1, s1 = conv2d_nhwc(x, b.conv1.weight, 1, 0, st)
    a1 = bn_act(y1, s1, b.bn1, True, training, group)
    y2, s2 = conv2d_nhwc(a1, b.conv2.weight, b.stride, 1, st)
    a2 = bn_act(y2, s2, b.bn2, True, training, group)
    y3, s3 = conv2d_nhwc(a2, b.conv3.weight, 1, 0, st)
    if len(b.shortcut) > 0:
        ys, ss = conv2d_nhwc(x, b.shortcut[0].weight, b.stride, 0, st)
        return bn_add_act(y3, s3, b.bn3, ys, ss, b.shortcut[1], None, training, group)
    return bn_add_act(y3, s3, b.bn3, x=x, training=training, group=group)


def _basic(b: BasicBlock, x, training, group):
    st = training
    y1, s1 = conv2d_nhwc(x, b.conv1.weight, b.stride, 1, st)
    a1 = bn_act(y1, s1, b.bn1, True, training, group)
    y2, s2 = conv2d_nhwc(a1, b.conv2.weight, 1, 1, st)
    if len(b.shortcut) > 0:
        ys, ss = conv2d_nhwc(x, b.shortcut[0].weight, b.stride, 0, st)
        return bn_add_act(y2, s2, b.bn2, ys, ss, b.shortcut[1], None, training, group)
    return bn_add_act(y2, s2, b.bn2, x=x, training=training, group=group)


def encoder_forward_native(enc: ResNet, x_nhwc: torch.Tensor, training: bool = True, group=None) -> torch.Tensor:
    """``x_nhwc``: [N, H, W, 8] bf16 (3 real channels). Returns fp32 [N, feat_dim]."""
    cin = enc.conv1.weight.shape[1]
    pad_c = x_nhwc.shape[-1] - cin
    if enc.stem == "cifar":      # 3x3/1, no max-pool (networks/resnet_big.py:75)
        y, s = conv2d_nhwc(x_nhwc, enc.conv1.weight, 1, 1, training, cin_pad=pad_c)
        out = bn_act(y, s, enc.bn1, True, training, group)
    else:                        # ImageNet stem: 7x7/2 conv + 3x3/2 max-pool
        y, s = conv2d_nhwc(x_nhwc, enc.conv1.weight, 2, 3, training, cin_pad=pad_c)
        out = maxpool_nhwc(bn_act(y, s, enc.bn1, True, training, group), 3, 2, 1)
    for blk in enc.blocks():
        if isinstance(blk, Bottleneck):
            out = _bottleneck(blk, out, training, group)
        else:
            out = _basic(blk, out, training, group)
    return global_avgpool_nhwc(out)


def head_forward(head, feat: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """Projection head in ``dtype`` with fp32 master weights (networks/resnet_big.py:168-172)."""
    if isinstance(head, torch.nn.Linear):
        return F.linear(feat.to(dtype), head.weight.to(dtype), head.bias.to(dtype)).float()
    l1, l2 = head[0], head[2]
    h = F.relu(F.linear(feat.to(dtype), l1.weight.to(dtype), l1.bias.to(dtype)))
    return F.linear(h, l2.weight.to(dtype), l2.bias.to(dtype)).float()


def to_nhwc_input(images: torch.Tensor, c_pad: int = INPUT_CHANNELS_PADDED) -> torch.Tensor:
    """NCHW float images -> NHWC bf16 with channels zero-padded to ``c_pad``."""
    x = images.permute(0, 2, 3, 1)
    if x.shape[-1] < c_pad:
        x = F.pad(x, (0, c_pad - x.shape[-1]))
    return x.to(torch.bfloat16).contiguous()


FUSED_HEAD = os.environ.get("SDX_FUSED_HEAD", "1") != "0"


class ModelRunner:
    """Runs a ``SupConResNet`` (or just its encoder) on the chosen backend.

    ``backend='torch'`` calls the modules (NCHW, autocast bf16 on GPU when requested);
    ``backend='native'`` uses the gfx950 kernels above. Inputs to :meth:`forward` are
    NCHW float images for ``torch`` and NHWC bf16 (C padded to 8) for ``native``.
    """

    def __init__(self, model, backend: str = "native", precision: str = "bf16", sync_group=None,
                 master: torch.Tensor = None, fused: bool = True):
        self.model = model
        self.backend = backend
        self.precision = precision
        self.sync_group = sync_group
        self.master = master
        self.fused = fused
        self._wc = None
        self._nbt = None
        # BatchNorm num_batches_tracked of the fused path: counted on the host and added to the
        # buffers when something reads them (state_dict: checkpoints, evaluation copies) — no
        # per-step kernel for a counter the training math never reads (momentum is set)
        self._nbt_pending = 0
        # flushed before any state_dict() / load_state_dict() that reaches a BN, called on the
        # top-level model or on any submodule (e.g. model.encoder): the hooks sit on every BN
        # module. A load flushes first, so the loaded counters replace the flushed ones instead
        # of having the pending count added on top later. Direct reads of
        # bn.num_batches_tracked between flushes see the last flushed value (the engines flush
        # at every epoch end).
        for m in model.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
                if hasattr(m, "register_state_dict_pre_hook"):
                    m.register_state_dict_pre_hook(lambda *a, **k: self.flush_bn_counters())
                if hasattr(m, "register_load_state_dict_pre_hook"):
                    m.register_load_state_dict_pre_hook(lambda *a, **k: self.flush_bn_counters())

    def weight_cache(self):
        if self._wc is None:
            from ..ops.weights import ConvWeightCache
            enc = self.model.encoder
            convs = [m for m in enc.modules() if isinstance(m, torch.nn.Conv2d)]
            head = getattr(self.model, "head", None)
            if head is not None:
                convs += [m for m in head.modules() if isinstance(m, torch.nn.Linear)]
            self._wc = ConvWeightCache(convs, self.master, {id(enc.conv1): INPUT_CHANNELS_PADDED})
            self._nbt = [m.num_batches_tracked for m in enc.modules()
                         if isinstance(m, torch.nn.BatchNorm2d) and m.num_batches_tracked is not None]
        return self._wc

    def prefetch_weights(self):
        """Start this step's bf16 weight conversion on the side stream (native fused path)."""
        if (self.backend == "native" and self.fused and self.master is not None
                and os.environ.get("SDX_WPREP_PREFETCH", "1") != "0"):
            self.weight_cache().prefetch()

    def _encode_fused(self, x, training):
        from ..ops import block as fb
        enc = self.model.encoder
        wc = self.weight_cache()
        wc.refresh()
        g = self.sync_group
        out = fb.stem(x, enc, wc, training, g)
        chain = fb.BlockChain()
        blocks = list(enc.blocks())
        for i, blk in enumerate(blocks):
            # every block but the last hands its output to a native block (forward BN3 fold)
            out = fb.bottleneck(out, blk, wc, training, g, chain, next_native=i + 1 < len(blocks)) \
                if isinstance(blk, Bottleneck) else fb.basic(out, blk, wc, training, g, chain)
        if training and self._nbt:
            self._nbt_pending += 1
        return global_avgpool_nhwc(out)

    def flush_bn_counters(self):
        """Add the host-counted training passes to every BN's num_batches_tracked."""
        if self._nbt_pending and self._nbt:
            torch._foreach_add_(self._nbt, self._nbt_pending)
        self._nbt_pending = 0

    def encode(self, x, training=None):
        enc = self.model.encoder
        training = enc.training if training is None else training
        if self.backend == "native":
            if self.fused:
                return self._encode_fused(x, training)
            return encoder_forward_native(enc, x, training, self.sync_group)
        if x.is_cuda and self.precision == "bf16":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return enc(x).float()
        return enc(x)

    def forward(self, x):
        feat = self.encode(x)
        if self.backend == "native" and self.fused and feat.is_cuda and FUSED_HEAD:
            from ..ops.head import projection_head
            return projection_head(feat, self.model.head, self.weight_cache())
        if self.backend == "native" or (x.is_cuda and self.precision == "bf16"):
            return head_forward(self.model.head, feat)
        return self.model.head(feat)
