"""Native linear evaluation (reference main_linear.py:166-244,
networks/resnet_big.py:196-204): the fused classifier + cross-entropy + top-k + SGD kernels
(csrc/kernels/linear_ce.hip) against fp32 torch (nn.Linear, F.cross_entropy, util.accuracy,
torch.optim.SGD), and the eval-mode encoder with BatchNorm folded into the convs against
the fp32 torch eval forward."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,C", [(2048, 10), (2048, 100), (512, 10)])
def test_linear_ce_matches_torch(gpu, K, C):
    from simclr_pytorch_distributed_amd.models.resnet import LinearClassifier
    from simclr_pytorch_distributed_amd.ops.linear_probe import NativeLinearCE
    from simclr_pytorch_distributed_amd.utils.meters import accuracy
    torch.manual_seed(K + C)
    name = "resnet50" if K == 2048 else "resnet18"
    nat = LinearClassifier(name, C).to(gpu)
    ref = LinearClassifier(name, C).to(gpu)
    ref.load_state_dict(nat.state_dict())
    opt = torch.optim.SGD(ref.parameters(), lr=5.0, momentum=0.9, weight_decay=1e-4)
    ce = NativeLinearCE(nat, momentum=0.9, weight_decay=1e-4)
    for step in range(3):
        B = 200 if step < 2 else 37                       # a partial last batch (drop_last=False)
        x = torch.randn(B, K, device=gpu).relu()
        y = torch.randint(0, C, (B,), device=gpu)
        lr = 5.0 * (0.5 ** step)
        for g in opt.param_groups:
            g["lr"] = lr
        out_t = ref(x)
        loss_t = F.cross_entropy(out_t, y)
        a1, a5 = accuracy(out_t, y, topk=(1, 5))
        out_n, st = ce.train_batch(x, y, lr)
        torch.cuda.synchronize()
        assert torch.allclose(out_n, out_t.detach(), rtol=1e-4, atol=1e-4)
        assert abs(float(st[0]) / B - float(loss_t)) <= 1e-4 * max(1.0, abs(float(loss_t)))
        assert abs(float(st[1]) * 100.0 / B - float(a1)) < 1e-3 and abs(float(st[2]) * 100.0 / B - float(a5)) < 1e-3
        opt.zero_grad()
        loss_t.backward()
        opt.step()
        assert torch.allclose(nat.fc.weight, ref.fc.weight, rtol=1e-5, atol=1e-6), step
        assert torch.allclose(nat.fc.bias, ref.fc.bias, rtol=1e-5, atol=1e-6), step
    out_e, st_e = ce.eval_batch(x, y)
    assert torch.allclose(out_e, ref(x).detach(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name", ["resnet50", "resnet18"])
def test_folded_eval_encoder(gpu, name):
    """Eval-mode encoder with BN folded into the convs (bias + ReLU epilogues, one
    elementwise pass per block output) vs the fp32 torch eval forward, on trained-looking BN
    statistics; bar: torch bf16 autocast's own error on the same input (x 1.5 + 1e-2)."""
    from simclr_pytorch_distributed_amd.models.executor import to_nhwc_input
    from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
    from simclr_pytorch_distributed_amd.ops.linear_probe import FoldedEncoder
    torch.manual_seed(1)
    m = SupConResNet(name).to(gpu).to(memory_format=torch.channels_last).eval()
    g = torch.Generator().manual_seed(2)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                c = mod.num_features
                mod.running_mean.copy_(0.2 * torch.randn(c, generator=g))
                mod.running_var.copy_(0.5 + torch.rand(c, generator=g))
                mod.weight.copy_(1 + 0.2 * torch.randn(c, generator=g))
                mod.bias.copy_(0.1 * torch.randn(c, generator=g))
    x = torch.randn(32, 3, 32, 32, generator=g).to(gpu).to(torch.bfloat16).float()
    with torch.no_grad():
        ref = m.encoder(x).float()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ac = m.encoder(x).float()
        got = FoldedEncoder(m.encoder)(to_nhwc_input(x))
    torch.cuda.synchronize()
    e_n = float((got - ref).norm() / ref.norm())
    e_c = float((ac - ref).norm() / ref.norm())
    print(f"{name} folded eval encoder rel error {e_n:.4g} (autocast {e_c:.4g})")
    assert got.shape == ref.shape
    assert e_n <= 1.5 * e_c + 1e-2


def test_linear_engine_native(gpu, tmp_path):
    """LinearEngine on the native path: folded encoder + fused classifier, a few steps and a
    validation pass on synthetic data; finite loss, accuracies in [0, 100]."""
    from simclr_pytorch_distributed_amd.config import parse_linear
    from simclr_pytorch_distributed_amd.engine.linear import LinearEngine
    opt = parse_linear(["--model", "resnet18", "--backend", "native", "--synthetic", "--synthetic_size", "512",
                        "--batch_size", "64", "--epochs", "1", "--max_steps", "3", "--learning_rate", "1",
                        "--work_dir", str(tmp_path)], make_dirs=True)
    eng = LinearEngine(opt, device=torch.device("cuda:0"))
    assert eng.folded is not None and eng.native_ce is not None
    loss, a1, a5 = eng.train_epoch(1)
    vl, v1, v5 = eng.validate()
    assert loss == loss and vl == vl
    assert 0.0 <= a1 <= 100.0 and 0.0 <= v1 <= v5 <= 100.0
