"""Metric helpers: :class:`AverageMeter` and top-k :func:`accuracy` (util.py:19-51),
plus :class:`DeviceMeter`, which accumulates on the GPU so the training step never
forces a host sync (the reference syncs 6x per step for logging)."""
from __future__ import annotations

import torch


class AverageMeter:
    """Computes and stores the average and current value."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def accuracy(output: torch.Tensor, target: torch.Tensor, topk=(1,)):
    """Top-k accuracy in percent, one 1-element tensor per k (util.py:37-51)."""
    with torch.no_grad():
        maxk = min(max(topk), output.size(1))
        batch_size = target.size(0)
        _, pred = output.topk(maxk, 1, True, True)
        pred = pred.t()
        correct = pred.eq(target.view(1, -1).expand_as(pred))
        res = []
        for k in topk:
            kk = min(k, maxk)
            correct_k = correct[:kk].reshape(-1).float().sum(0, keepdim=True)
            res.append(correct_k.mul_(100.0 / batch_size))
        return res


class DeviceMeter:
    """Running sum/count kept as device tensors; ``.val``/``.avg`` sync only when read."""

    def __init__(self, device=None):
        self.device = device
        self.reset()

    def reset(self):
        self._sum = None
        self._last = None
        self.count = 0

    def update(self, val: torch.Tensor, n: int = 1):
        v = val.detach().float().reshape(())
        self._last = v
        self._sum = v * n if self._sum is None else self._sum + v * n
        self.count += n

    @property
    def val(self) -> float:
        return 0.0 if self._last is None else float(self._last)

    @property
    def avg(self) -> float:
        return 0.0 if self._sum is None else float(self._sum) / max(self.count, 1)
