"""Checkpoint layout, safe loading, resume and pretrain -> linear-probe round trip (CPU).

Reference layout (util.py:87-96): {'opt', 'model', 'optimizer', 'epoch'} with DDP
``module.``-prefixed model keys (322 for SupConResNet-50).
"""
import argparse
import os

import pytest
import torch


def _pre_opt(tmp_path, extra=()):
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    return parse_pretrain(["--model", "resnet18", "--batch_size", "8", "--synthetic", "--synthetic_size", "32",
                           "--epochs", "2", "--save_freq", "1", "--print_freq", "100", "--backend", "torch",
                           "--work_dir", str(tmp_path / "ws"), *extra], make_dirs=True)


def test_layout_and_prefix(tmp_path):
    from simclr_pytorch_distributed_amd.engine import checkpoint as ck
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    m = SupConResNet("resnet50")
    o = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    f = str(tmp_path / "c.pth")
    ck.save_model(m, o, argparse.Namespace(lr=0.1, model="resnet50"), 3, f)
    st = ck.load_checkpoint(f)
    assert set(st) == {"opt", "model", "optimizer", "epoch"}
    assert st["epoch"] == 3 and st["opt"]["model"] == "resnet50"
    assert len(st["model"]) == 322 and all(k.startswith("module.") for k in st["model"])
    m2 = SupConResNet("resnet50")
    ck.load_model_state(m2, st["model"])
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k


def test_reference_style_checkpoint_loads_safely(tmp_path):
    """A checkpoint written the reference way (pickled argparse.Namespace) loads through the
    weights_only=True path with an allow-list — no unrestricted unpickling."""
    from simclr_pytorch_distributed_amd.engine import checkpoint as ck
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    m = SupConResNet("resnet18")
    sd = {"module." + k: v for k, v in m.state_dict().items()}
    f = str(tmp_path / "ref.pth")
    torch.save({"opt": argparse.Namespace(model="resnet18", temp=0.5), "model": sd, "optimizer": {}, "epoch": 100}, f)
    st = ck.load_checkpoint(f)
    assert st["epoch"] == 100 and st["opt"].model == "resnet18"
    m2 = SupConResNet("resnet18")
    ck.load_model_state(m2, st["model"])


def test_strict_mismatch_raises():
    from simclr_pytorch_distributed_amd.engine import checkpoint as ck
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    with pytest.raises(KeyError):
        ck.load_model_state(SupConResNet("resnet18"), SupConResNet("resnet50").state_dict())


def test_resume_restores_model_optimizer_epoch(tmp_path):
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    opt = _pre_opt(tmp_path, ["--max_steps", "2"])
    eng = PretrainEngine(opt, device=torch.device("cpu"))
    last = eng.run()
    assert os.path.exists(last) and os.path.exists(os.path.join(opt.save_folder, "ckpt_epoch_1.pth"))
    w = eng.flat.flat.clone()
    mom = eng.optimizer.state_dict()
    opt2 = _pre_opt(tmp_path, ["--max_steps", "2", "--resume", os.path.join(opt.save_folder, "ckpt_epoch_1.pth")])
    eng2 = PretrainEngine(opt2, device=torch.device("cpu"))
    assert eng2.start_epoch == 2 and eng2.global_step == 2
    opt3 = _pre_opt(tmp_path, ["--resume", last])
    eng3 = PretrainEngine(opt3, device=torch.device("cpu"))
    assert eng3.start_epoch == 3
    assert torch.equal(eng3.flat.flat, w)
    s3 = eng3.optimizer.state_dict()
    for k in mom["state"]:
        assert torch.equal(s3["state"][k]["momentum_buffer"], mom["state"][k]["momentum_buffer"])


def test_pretrain_to_linear_round_trip(tmp_path):
    from simclr_pytorch_distributed_amd.config import parse_linear
    from simclr_pytorch_distributed_amd.engine.linear import LinearEngine
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    opt = _pre_opt(tmp_path, ["--max_steps", "1", "--epochs", "1"])
    eng = PretrainEngine(opt, device=torch.device("cpu"))
    last = eng.run()
    lopt = parse_linear(["--model", "resnet18", "--batch_size", "8", "--synthetic", "--synthetic_size", "32",
                         "--epochs", "1", "--max_steps", "1", "--backend", "torch", "--ckpt", last,
                         "--work_dir", str(tmp_path / "lin")], make_dirs=True)
    le = LinearEngine(lopt, device=torch.device("cpu"))
    for (k, a), (_, b) in zip(eng.model.encoder.state_dict().items(), le.model.encoder.state_dict().items()):
        assert torch.equal(a.cpu(), b.cpu()), k
    best, best5 = le.run()
    assert 0.0 <= best <= 100.0
