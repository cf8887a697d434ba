"""CLI parity with the reference parsers (main_supcon.py:22-152, main_linear.py:21-116)."""
import datetime
import math

from simclr_pytorch_distributed_amd.config import parse_linear, parse_pretrain, pretrain_parser

NOW = datetime.datetime(2026, 10, 15, 21, 5)


def test_pretrain_defaults(tmp_path):
    o = parse_pretrain(["--work_dir", str(tmp_path)], make_dirs=False, now=NOW)
    assert (o.print_freq, o.save_freq, o.batch_size, o.num_workers, o.epochs) == (10, 20, 256, 16, 1000)
    assert (o.learning_rate, o.lr_decay_rate, o.weight_decay, o.momentum) == (0.5, 0.1, 1e-4, 0.9)
    assert o.lr_decay_epochs == [700, 800, 900]
    assert (o.model, o.dataset, o.size, o.method, o.temp) == ("resnet50", "cifar10", 32, "SimCLR", 0.5)
    assert (o.cosine, o.syncBN, o.warm, o.trial, o.sec, o.l2reg) == (False, False, False, "0", False, False)
    assert (o.sec_wei, o.norm_momentum, o.l2reg_wei, o.ckpt) == (0.0, 1.0, 0.0, "")
    assert o.model_name == "SimCLR_cifar10_resnet50_lr_0.5_decay_0.0001_bsz_256_temp_0.5_trial_0"
    assert o.save_folder.endswith("cifar10_models/cifar10_1015_2105_" + o.model_name)
    assert o.tb_folder.endswith("cifar10_tensorboard/cifar10_1015_2105_" + o.model_name)
    assert o.record_norm_mean is None


def test_pretrain_derived_warm_cosine(tmp_path):
    o = parse_pretrain(["--batch_size", "1024", "--cosine", "--sec", "--epochs", "100", "--work_dir", str(tmp_path)],
                       make_dirs=False, now=NOW)
    assert o.warm and o.model_name.endswith("_cosine_sec_warm")
    eta_min = 0.5 * 0.1 ** 3
    assert abs(o.warmup_to - (eta_min + (0.5 - eta_min) * (1 + math.cos(math.pi * 10 / 100)) / 2)) < 1e-12
    assert o.warmup_from == 0.01 and o.warm_epochs == 10


def test_local_rank_aliases(tmp_path):
    p = pretrain_parser()
    assert p.parse_args(["--local_rank", "1"]).local_rank == 1
    assert p.parse_args(["--local-rank=3"]).local_rank == 3


def test_path_dataset_safe_parse(tmp_path):
    o = parse_pretrain(["--dataset", "path", "--data_folder", str(tmp_path), "--mean", "(0.1, 0.2, 0.3)",
                        "--std", "(0.4,0.5,0.6)", "--work_dir", str(tmp_path)], make_dirs=False, now=NOW)
    assert o.mean_t == (0.1, 0.2, 0.3) and o.std_t == (0.4, 0.5, 0.6)


def test_linear_defaults(tmp_path):
    o = parse_linear(["--work_dir", str(tmp_path)], make_dirs=False, now=NOW)
    assert (o.batch_size, o.epochs, o.learning_rate, o.lr_decay_rate, o.weight_decay) == (512, 100, 0.1, 0.2, 0)
    assert o.lr_decay_epochs == [60, 75, 90] and o.n_cls == 10
    assert o.model_name == "cifar10_resnet50_lr_0.1_decay_0_bsz_512"
    assert "classifier_1015_2105_" in o.save_folder


def test_run_folder_collision_guard(tmp_path):
    a = parse_pretrain(["--work_dir", str(tmp_path)], now=NOW)
    b = parse_pretrain(["--work_dir", str(tmp_path)], now=NOW)
    assert a.save_folder != b.save_folder
