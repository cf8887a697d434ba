"""LR schedules are value-identical to util.py:54-76."""
import math
from types import SimpleNamespace

import torch

from simclr_pytorch_distributed_amd.optim.schedules import adjust_learning_rate, lr_at_epoch, warmup_learning_rate


def _opt():
    return torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=0.0)


def test_cosine_epoch1():
    a = SimpleNamespace(learning_rate=0.5, cosine=True, lr_decay_rate=0.1, epochs=100, lr_decay_epochs=[])
    o = _opt()
    lr = adjust_learning_rate(a, o, 1)
    assert abs(lr - 0.49988) < 1e-5 and o.param_groups[0]["lr"] == lr
    # last epoch reaches eta_min
    assert abs(lr_at_epoch(a, 100) - 0.5 * 0.1 ** 3) < 1e-12


def test_step_schedule():
    a = SimpleNamespace(learning_rate=5.0, cosine=False, lr_decay_rate=0.2, epochs=100,
                        lr_decay_epochs=[60, 75, 90])
    assert lr_at_epoch(a, 60) == 5.0
    assert abs(lr_at_epoch(a, 61) - 1.0) < 1e-12
    assert abs(lr_at_epoch(a, 91) - 5.0 * 0.2 ** 3) < 1e-12


def test_warmup():
    a = SimpleNamespace(warm=True, warm_epochs=10, warmup_from=0.01, warmup_to=0.5)
    o = _opt()
    lr = warmup_learning_rate(a, 1, 0, 100, o)
    assert abs(lr - 0.01) < 1e-12
    lr = warmup_learning_rate(a, 10, 99, 100, o)
    assert abs(lr - (0.01 + (999 / 1000) * 0.49)) < 1e-12
    assert warmup_learning_rate(a, 11, 0, 100, o) is None
