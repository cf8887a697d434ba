"""Gradient-cache micro-batching (``--micro_batch``): with batch-independent layers (BN in
eval mode) the chunked encoder passes must reproduce the full-batch step exactly, and in
train mode the step must run with the loss of the full batch."""
import torch


def _engine(tmp_path, mb, seed=0):
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    opt = parse_pretrain(["--model", "resnet18", "--batch_size", "8", "--synthetic", "--synthetic_size", "32",
                          "--epochs", "1", "--backend", "torch", "--learning_rate", "0.1", "--seed", str(seed),
                          "--micro_batch", str(mb), "--work_dir", str(tmp_path / f"mb{mb}")], make_dirs=False)
    return PretrainEngine(opt, device=torch.device("cpu"))


def test_gradcache_equals_full_batch_with_eval_bn(tmp_path):
    a, b = _engine(tmp_path, 0), _engine(tmp_path, 4)
    b.model.load_state_dict(a.model.state_dict())
    for e in (a, b):
        e.model.train()
        for m in e.model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.eval()
    idx = torch.arange(8)
    sa = a.train_step(idx, 1, 0, 4)
    sb = b.train_step(idx, 1, 0, 4)
    assert torch.allclose(sa["loss_local"], sb["loss_local"], rtol=1e-5)
    assert torch.allclose(a.flat.flat, b.flat.flat, rtol=1e-4, atol=1e-6)


def test_gradcache_train_mode_runs(tmp_path):
    e = _engine(tmp_path, 4)
    e.model.train()
    before = e.flat.flat.clone()
    rm0 = e.model.encoder.bn1.running_mean.clone()
    st = e.train_step(torch.arange(8), 1, 0, 4)
    assert torch.isfinite(st["loss_local"])
    assert not torch.equal(before, e.flat.flat)
    # running stats: updated by the re-encode pass only (4 chunks of 4 views)
    assert int(e.model.encoder.bn1.num_batches_tracked) == 4
    assert not torch.equal(rm0, e.model.encoder.bn1.running_mean)


def test_gradcache_train_mode_is_exact_ghost_batchnorm(tmp_path, monkeypatch):
    """The documented train-mode semantics of --micro_batch V: the update is the EXACT
    gradient of the full-batch loss of a network whose BatchNorms normalise each chunk of V
    views with that chunk's statistics (ghost batch norm), and the running statistics take
    one momentum update per chunk. Reference: the full batch in ONE autograd pass with every
    BatchNorm2d.forward split into V-view chunks (same views, same order)."""
    import torch.nn.functional as F
    V = 4
    a, b = _engine(tmp_path, V), _engine(tmp_path, 0)
    b.model.load_state_dict(a.model.state_dict())
    a.model.train()
    b.model.train()
    orig = torch.nn.BatchNorm2d.forward

    def ghost(self, x):
        outs = []
        for c in torch.split(x, V):
            self.num_batches_tracked.add_(1)
            outs.append(F.batch_norm(c, self.running_mean, self.running_var, self.weight, self.bias, True,
                                     self.momentum, self.eps))
        return torch.cat(outs)

    idx = torch.arange(8)
    sa = a.train_step(idx, 1, 0, 4)
    monkeypatch.setattr(torch.nn.BatchNorm2d, "forward", ghost)
    sb = b.train_step(idx, 1, 0, 4)
    monkeypatch.setattr(torch.nn.BatchNorm2d, "forward", orig)
    assert torch.allclose(sa["loss_local"], sb["loss_local"], rtol=1e-5)
    assert torch.allclose(a.flat.flat, b.flat.flat, rtol=1e-4, atol=1e-6)
    ra, rb = a.model.encoder.bn1, b.model.encoder.bn1
    assert torch.allclose(ra.running_mean, rb.running_mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(ra.running_var, rb.running_var, rtol=1e-5, atol=1e-6)
    assert int(ra.num_batches_tracked) == int(rb.num_batches_tracked) == 16 // V
