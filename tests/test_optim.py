"""Flat-buffer optimizers: torch fallback path == torch.optim.SGD; state-dict round trip."""
import torch

from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
from simclr_pytorch_distributed_amd.optim.flat import FlatParams, FusedLARS, FusedSGD


def _tiny():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.Flatten(),
                               torch.nn.Linear(8 * 6 * 6, 4))


def test_fused_sgd_matches_torch_sgd():
    a, b = _tiny(), _tiny()
    b.load_state_dict(a.state_dict())
    flat = FlatParams(a)
    oa = FusedSGD(flat, lr=1e-3, momentum=0.9, weight_decay=1e-3, backend="torch")
    ob = torch.optim.SGD(b.parameters(), lr=1e-3, momentum=0.9, weight_decay=1e-3)
    x = torch.randn(5, 3, 8, 8)
    for step in range(4):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            m(x).tanh().sum().backward()
            o.step()
        oa.param_groups[0]["lr"] = ob.param_groups[0]["lr"] = 1e-3 / (step + 2)
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.allclose(p, q, atol=1e-6)
    sd = oa.state_dict()
    ref = ob.state_dict()
    for i in ref["state"]:
        assert torch.allclose(sd["state"][i]["momentum_buffer"], ref["state"][i]["momentum_buffer"], atol=1e-6)


def test_flat_views_keep_channels_last():
    m = SupConResNet("resnet18").to(memory_format=torch.channels_last)
    flat = FlatParams(m)
    w = m.encoder.layer1[0].conv1.weight
    assert w.is_contiguous(memory_format=torch.channels_last)
    assert w.data_ptr() >= flat.flat.data_ptr()
    assert flat.total % 4096 == 0


def test_lars_runs_and_excludes_bn():
    m = _tiny()
    flat = FlatParams(m)
    o = FusedLARS(flat, lr=1.0, momentum=0.9, weight_decay=1e-4, backend="torch")
    before = [p.detach().clone() for p in m.parameters()]
    m(torch.randn(4, 3, 8, 8)).sum().backward()
    o.step()
    assert all(not torch.equal(p, q) for p, q in zip(m.parameters(), before))
