"""Small-component parity checks on CPU."""
import logging
import os

import torch
import torch.nn as nn


def test_accuracy_and_average_meter():
    """util.py:19-51: AverageMeter running mean; accuracy() top-k in percent."""
    from simclr_pytorch_distributed_amd.utils.meters import AverageMeter, accuracy
    m = AverageMeter()
    for v, n in ((1.0, 2), (4.0, 1)):
        m.update(v, n)
    assert m.val == 4.0 and m.count == 3 and abs(m.avg - 2.0) < 1e-12
    out = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.15, 0.05], [0.2, 0.3, 0.5], [0.5, 0.3, 0.2]])
    tgt = torch.tensor([1, 1, 0, 2])
    a1, a2 = accuracy(out, tgt, topk=(1, 2))
    assert abs(a1.item() - 25.0) < 1e-6          # only row 0 right at top-1
    assert abs(a2.item() - 50.0) < 1e-6          # rows 0, 1 within top-2


def test_linear_batchnorm_equals_bn1d():
    """networks/resnet_big.py:145-156: BN1d implemented through BN2d."""
    from simclr_pytorch_distributed_amd.models.resnet import LinearBatchNorm
    torch.manual_seed(0)
    lb, ref = LinearBatchNorm(16), nn.BatchNorm1d(16)
    x = torch.randn(8, 16)
    assert torch.allclose(lb(x), ref(x), atol=1e-6)
    assert torch.allclose(lb.bn.running_mean, ref.running_mean, atol=1e-6)


def test_model_dict_and_classifiers():
    """networks/resnet_big.py:137-142, 184-204: registry dims, SupCEResNet, LinearClassifier."""
    from simclr_pytorch_distributed_amd.models.resnet import LinearClassifier, model_dict
    assert {k: v[1] for k, v in model_dict.items()} == {"resnet18": 512, "resnet34": 512, "resnet50": 2048,
                                                      "resnet101": 2048}
    lc = LinearClassifier("resnet50", 100)
    assert lc(torch.randn(3, 2048)).shape == (3, 100)


def test_file_logger_writes_log_ing(tmp_path):
    """util.py:98-114: rank 0 logs to <save_folder>/log-ing."""
    from simclr_pytorch_distributed_amd.utils.logging import setup_logging
    before = list(logging.root.handlers)
    try:
        setup_logging(str(tmp_path), 0)
        logging.info("parity-check-line")
        for h in logging.root.handlers:
            h.flush()
        path = os.path.join(tmp_path, "log-ing")
        assert os.path.exists(path)
        assert "parity-check-line" in open(path).read()
    finally:
        for h in list(logging.root.handlers):
            if h not in before:
                logging.root.removeHandler(h)
                h.close()


def test_sec_l2reg_terms_cpu(tmp_path):
    """main_supcon.py:295-317: SEC / L2-reg regularisers enter the loss, the EMA record of the
    feature-norm mean is initialised from the first batch (norm_momentum 1.0 = no EMA)."""
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    opt = parse_pretrain(["--batch_size", "8", "--synthetic", "--synthetic_size", "32", "--work_dir", str(tmp_path),
                          "--model", "resnet18", "--backend", "torch", "--sec", "--sec_wei", "0.5", "--l2reg",
                          "--l2reg_wei", "0.1", "--epochs", "2"], make_dirs=False)
    eng = PretrainEngine(opt)
    st = eng.train_step(torch.arange(8), 1, 3, 4)
    for k in ("norm_mean", "norm_var", "loss_sec", "loss_l2reg", "record_norm_mean"):
        assert torch.isfinite(torch.as_tensor(st[k])).all()
    assert float(st["loss_l2reg"]) > 0
    assert abs(float(st["record_norm_mean"]) - float(st["norm_mean"])) < 1e-5
