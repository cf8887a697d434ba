"""Native linear evaluation (reference main_linear.py:119-244,
networks/resnet_big.py:196-204).

* :class:`FoldedEncoder` — the frozen encoder in eval mode with every BatchNorm folded into
  its conv: W' = W·γ/√(σ²+ε) per output channel, b' = β − μ·γ/√(σ²+ε). Each conv (+BN +ReLU)
  is ONE implicit-GEMM launch whose epilogue adds b' (and applies the ReLU) on the fp32
  accumulators before the bf16 rounding; a block output is relu(y3' + shortcut) in one
  elementwise pass. No BatchNorm kernel runs at all. The encoder is frozen for the whole
  probe, so the fold is computed once.
* :class:`NativeLinearCE` — ``LinearClassifier`` + ``CrossEntropyLoss`` + top-1/5 +
  ``torch.optim.SGD`` as two fused launches per batch (csrc/kernels/linear_ce.hip), fp32 as
  the reference classifier; the statistics stay on the device.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from . import _ext
from .pool import global_avgpool_nhwc, maxpool_nhwc
from ..models.resnet import Bottleneck


def _fold(conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, c_pad: int = 0):
    """bf16 KRSC weights and fp32 bias of conv followed by eval-mode bn."""
    w = conv.weight.detach().float()
    inv = torch.rsqrt(bn.running_var.float() + bn.eps)
    g = bn.weight.detach().float() if bn.weight is not None else torch.ones_like(inv)
    b = bn.bias.detach().float() if bn.bias is not None else torch.zeros_like(inv)
    scale = g * inv
    wk = (w * scale[:, None, None, None]).permute(0, 2, 3, 1)            # [K][R][S][C]
    if c_pad > wk.shape[-1]:
        wk = torch.nn.functional.pad(wk, (0, c_pad - wk.shape[-1]))
    bias = (b - bn.running_mean.float() * scale).contiguous()
    return wk.to(torch.bfloat16).contiguous(), bias


class FoldedEncoder:
    """Eval-mode native forward of a ``models.resnet.ResNet`` with folded BatchNorm."""

    def __init__(self, enc, c_pad: int = 8):
        self.enc = enc
        self.stem = getattr(enc, "stem", "cifar")
        self.w0, self.b0 = _fold(enc.conv1, enc.bn1, c_pad)
        self.blocks: List[Dict] = []
        for blk in enc.blocks():
            d: Dict = {"bottle": isinstance(blk, Bottleneck), "stride": blk.stride}
            d["c1"] = _fold(blk.conv1, blk.bn1)
            d["c2"] = _fold(blk.conv2, blk.bn2)
            if d["bottle"]:
                d["c3"] = _fold(blk.conv3, blk.bn3)
            d["sc"] = _fold(blk.shortcut[0], blk.shortcut[1]) if len(blk.shortcut) > 0 else None
            self.blocks.append(d)
        dev = self.b0.device
        self._ones, self._zeros = {}, {}
        for d in self.blocks:
            c = (d["c3"] if d["bottle"] else d["c2"])[1].numel()
            self._ones.setdefault(c, torch.ones(c, device=dev))
            self._zeros.setdefault(c, torch.zeros(c, device=dev))

    @torch.no_grad()
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        """``x``: NHWC bf16 [N, H, W, 8] -> fp32 features [N, feat_dim]."""
        m = _ext.require()
        if self.stem == "cifar":
            out = m.conv_fwd_bias(x, self.w0, 1, 1, self.b0, True)
        else:
            out = maxpool_nhwc(m.conv_fwd_bias(x, self.w0, 2, 3, self.b0, True), 3, 2, 1)
        for d in self.blocks:
            st = d["stride"]
            if d["bottle"]:
                a1 = m.conv_fwd_bias(out, d["c1"][0], 1, 0, d["c1"][1], True)
                a2 = m.conv_fwd_bias(a1, d["c2"][0], st, 1, d["c2"][1], True)
                y = m.conv_fwd_bias(a2, d["c3"][0], 1, 0, d["c3"][1], False)
            else:
                a1 = m.conv_fwd_bias(out, d["c1"][0], st, 1, d["c1"][1], True)
                y = m.conv_fwd_bias(a1, d["c2"][0], 1, 1, d["c2"][1], False)
            sc = m.conv_fwd_bias(out, d["sc"][0], st, 0, d["sc"][1], False) if d["sc"] is not None else out
            c = y.shape[-1]
            out = m.bn_apply(y, self._ones[c], self._zeros[c], sc, None, None, 2, True, None)   # relu(y + sc)
        return global_avgpool_nhwc(out)


class NativeLinearCE:
    """``LinearClassifier`` trained with cross-entropy and SGD on the native path. Holds its
    own momentum buffers (the linear probe writes no checkpoint, main_linear.py)."""

    def __init__(self, classifier: torch.nn.Module, momentum: float = 0.9, weight_decay: float = 0.0):
        fc = classifier.fc
        self.W, self.b = fc.weight, fc.bias
        self.momentum = float(momentum)
        self.weight_decay = float(weight_decay)
        self.bufW = torch.zeros_like(self.W)
        self.bufb = torch.zeros_like(self.b)
        self.first = True

    def train_batch(self, feats: torch.Tensor, labels: torch.Tensor, lr: float):
        """One SGD step on the batch; returns (logits, stats [Σ CE, hits@1, hits@5]) on device."""
        with torch.no_grad():
            out = _ext.require().linear_ce_step(feats.float().contiguous(), self.W.data, self.b.data, labels.long(),
                                                self.bufW, self.bufb, float(lr), self.momentum, self.weight_decay,
                                                self.first, True)
        self.first = False
        return out[0], out[1]

    @torch.no_grad()
    def eval_batch(self, feats: torch.Tensor, labels: torch.Tensor):
        out = _ext.require().linear_ce_step(feats.float().contiguous(), self.W.data, self.b.data, labels.long(),
                                            None, None, 0.0, 0.0, 0.0, False, False)
        return out[0], out[1]


def supported(classifier: torch.nn.Module, feat_dim: Optional[int] = None) -> bool:
    fc = getattr(classifier, "fc", None)
    if fc is None or not fc.weight.is_cuda or not _ext.available():
        return False
    k, c = fc.in_features, fc.out_features
    return k % 64 == 0 and k <= 2048 and ((k // 64) & (k // 64 - 1)) == 0 and c <= 1024
