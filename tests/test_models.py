"""Model structure parity (networks/resnet_big.py) — counts measured on the reference."""
import pytest
import torch

from simclr_pytorch_distributed_amd.models.resnet import LinearClassifier, SupCEResNet, SupConResNet

COUNTS = {"resnet18": (11497152, 11168832, 20), "resnet34": (21605312, 21276992, 36),
          "resnet50": (27958976, 23500352, 53), "resnet101": (46951104, 42492480, 104)}


@pytest.mark.parametrize("name", list(COUNTS))
def test_param_counts(name):
    m = SupConResNet(name)
    total, enc, nbn = COUNTS[name]
    assert sum(p.numel() for p in m.parameters()) == total
    assert sum(p.numel() for p in m.encoder.parameters()) == enc
    assert sum(isinstance(x, torch.nn.BatchNorm2d) for x in m.modules()) == nbn


def test_state_dict_keys_match_reference_layout():
    sd = SupConResNet("resnet50").state_dict()
    assert len(sd) == 322
    assert "encoder.layer1.0.shortcut.0.weight" in sd and "encoder.layer4.2.bn3.num_batches_tracked" in sd
    assert "head.0.weight" in sd and "head.2.bias" in sd


def test_forward_shapes():
    m = SupConResNet("resnet18")
    assert m(torch.randn(2, 3, 32, 32)).shape == (2, 128)
    assert SupConResNet("resnet18", head="linear")(torch.randn(2, 3, 32, 32)).shape == (2, 128)
    assert SupCEResNet("resnet18", 10)(torch.randn(2, 3, 32, 32)).shape == (2, 10)
    assert LinearClassifier("resnet50", 100)(torch.randn(2, 2048)).shape == (2, 100)
    assert SupConResNet("resnet18", stem="imagenet")(torch.randn(2, 3, 64, 64)).shape == (2, 128)


def test_host_counted_bn_passes_flush_on_submodule_state_dict_and_load():
    """The native runner counts BN training passes on the host (models/executor.py): a
    state_dict() of a SUBMODULE flushes them, and a load_state_dict() flushes first so the
    loaded counters replace them instead of having the pending count added later."""
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    m = SupConResNet("resnet18")
    r = ModelRunner(m, "native", fused=True)
    r._nbt = [b.num_batches_tracked for b in m.encoder.modules() if isinstance(b, torch.nn.BatchNorm2d)]
    r._nbt_pending = 3
    sd = {k: v.clone() for k, v in m.encoder.state_dict().items()}
    assert int(sd["bn1.num_batches_tracked"]) == 3 and r._nbt_pending == 0
    r._nbt_pending = 2
    sd["bn1.num_batches_tracked"].fill_(7)
    m.encoder.load_state_dict(sd)
    assert r._nbt_pending == 0
    assert int(m.encoder.bn1.num_batches_tracked) == 7
    assert int(m.state_dict()["encoder.bn1.num_batches_tracked"]) == 7
