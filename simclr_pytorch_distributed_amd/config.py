"""Command-line configuration with flag/default/derived-field parity to the reference.

* :func:`pretrain_parser` / :func:`parse_pretrain` mirror main_supcon.py:22-152
  (30 flags, ``model_name`` derivation, warm-up auto-enable for ``batch_size > 256``,
  ``./work_space/{dataset}_{models,tensorboard}/{dataset}_{MMDD_HHMM}_{model_name}``).
* :func:`linear_parser` / :func:`parse_linear` mirror main_linear.py:21-116.

Additions (new flags only; no reference flag changes meaning):
``--local-rank`` (dashed alias), env rank discovery (Q13),
``--precision``, ``--backend``, ``--synthetic``, ``--stem``, ``--optimizer {sgd,lars}``,
``--grad_semantics {ref,exact}`` (Q2), ``--dist_backend``, ``--seed``, ``--head``,
``--feat_dim`` (Q11), ``--resume``, ``--cuda_graph``, ``--work_dir``.
Fixes: ``--num_workers`` is honoured (Q6): it sizes the image-decode thread pool of
``dataset=path`` and the CPU augmentation threads of ``--gpu_aug 0`` (the default pipeline
is the GPU kernel, which needs no workers); ``dataset=path`` parses ``--mean/--std``
safely and uses the std (Q5); run folders get a collision guard (Q21).
"""
from __future__ import annotations

import argparse
import ast
import datetime
import math
import os
from typing import List, Optional, Sequence

DATASET_STATS = {
    # main_supcon.py:157-162 / main_ce.py:21-26
    "cifar10": ((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)),
    "cifar100": ((0.5071, 0.4867, 0.4408), (0.2675, 0.2565, 0.2761)),
}
N_CLASSES = {"cifar10": 10, "cifar100": 100}


def parse_tuple(s: Optional[str]):
    """Parse ``"(0.5, 0.5, 0.5)"`` without ``eval`` (reference uses eval, main_supcon.py:164)."""
    if s is None:
        return None
    v = ast.literal_eval(s)
    if isinstance(v, (int, float)):
        return (float(v),)
    return tuple(float(x) for x in v)


def env_rank_info(cli_local_rank: Optional[int] = None):
    """Return (rank, local_rank, world_size) from torchrun env vars, falling back to the CLI."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = os.environ.get("LOCAL_RANK")
    local_rank = int(local) if local is not None else (cli_local_rank or 0)
    if "RANK" not in os.environ and cli_local_rank:
        rank = cli_local_rank
    return rank, local_rank, world


def _add_common_new_flags(p: argparse.ArgumentParser):
    g = p.add_argument_group("MI355X framework options (new)")
    g.add_argument("--backend", type=str, default="auto", choices=["auto", "native", "torch"],
                   help="compute path: native gfx950 kernels, stock torch ops, or auto")
    g.add_argument("--precision", type=str, default="bf16", choices=["bf16", "fp32"],
                   help="activation/compute dtype on GPU (fp32 master weights always)")
    g.add_argument("--synthetic", action="store_true", help="use synthetic data (no dataset files)")
    g.add_argument("--synthetic_size", type=int, default=50000)
    g.add_argument("--seed", type=int, default=0)
    g.add_argument("--stem", type=str, default="cifar", choices=["cifar", "imagenet"])
    g.add_argument("--head", type=str, default="mlp", choices=["mlp", "linear"])
    g.add_argument("--feat_dim", type=int, default=128)
    g.add_argument("--work_dir", type=str, default="./work_space")
    g.add_argument("--dist_backend", type=str, default="auto", choices=["auto", "nccl", "gloo"])
    g.add_argument("--cuda_graph", action="store_true", help="capture the train step in a HIP graph")
    g.add_argument("--max_steps", type=int, default=0, help="stop each epoch after this many steps (0 = all)")
    g.add_argument("--gpu_aug", type=int, default=1,
                   help="augmentation on the GPU kernel (1) or the CPU torch pipeline on --num_workers threads (0)")
    # default rccl: the fused xGMI exchange has only ever run as same-device IPC
    # rehearsals (several processes on one GPU, emulated ranks); its peer stores and flag
    # protocol have not yet executed across real xGMI links, so it is opt-in until they have
    g.add_argument("--syncbn_comm", type=str, default="rccl", choices=["auto", "rccl", "xgmi"],
                   help="SyncBN statistics exchange: rccl (default: a dedicated RCCL communicator, "
                        "reduce -> ncclAllReduce -> finalize per BN), xgmi (the fused one-shot xGMI exchange, "
                        "every rank on one node; RCCL is the fallback when the arena's self-check fails), "
                        "auto (set up both and keep the one measured fastest on the first batch, agreed by "
                        "all ranks). xgmi/auto are EXPERIMENTAL: the fused exchange has been validated on "
                        "one GPU (multi-process IPC rehearsals, emulated ranks) but not yet across real "
                        "peer GPUs")
    g.add_argument("--comm_timeout", type=float, default=600.0,
                   help="collective timeout in seconds (a dead/stalled peer raises instead of hanging)")
    g.add_argument("--profile", action="store_true",
                   help="per-phase HIP-event timings in the log + ROCTX ranges for rocprofv3 --marker-trace")


def pretrain_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("argument for training")
    # main_supcon.py:26-34
    p.add_argument("--print_freq", type=int, default=10, help="print frequency")
    p.add_argument("--save_freq", type=int, default=20, help="save frequency")
    p.add_argument("--batch_size", type=int, default=256, help="batch_size (global)")
    p.add_argument("--num_workers", type=int, default=16, help="num of workers to use")
    p.add_argument("--epochs", type=int, default=1000, help="number of training epochs")
    # optimization (main_supcon.py:37-46)
    p.add_argument("--learning_rate", type=float, default=0.5, help="learning rate")
    p.add_argument("--lr_decay_epochs", type=str, default="700,800,900", help="where to decay lr")
    p.add_argument("--lr_decay_rate", type=float, default=0.1, help="decay rate for learning rate")
    p.add_argument("--weight_decay", type=float, default=1e-4, help="weight decay")
    p.add_argument("--momentum", type=float, default=0.9, help="momentum")
    # model dataset (main_supcon.py:49-56)
    p.add_argument("--model", type=str, default="resnet50")
    p.add_argument("--dataset", type=str, default="cifar10", choices=["cifar10", "cifar100", "path"])
    p.add_argument("--mean", type=str, help="mean of dataset in path in form of str tuple")
    p.add_argument("--std", type=str, help="std of dataset in path in form of str tuple")
    p.add_argument("--data_folder", type=str, default=None, help="path to custom dataset")
    p.add_argument("--size", type=int, default=32, help="parameter for RandomResizedCrop")
    # method / temperature (main_supcon.py:59-63)
    p.add_argument("--method", type=str, default="SimCLR", choices=["SupCon", "SimCLR"])
    p.add_argument("--temp", type=float, default=0.5, help="temperature for loss function")
    # other (main_supcon.py:66-88)
    p.add_argument("--cosine", action="store_true", help="using cosine annealing")
    p.add_argument("--syncBN", action="store_true", help="using synchronized batch normalization")
    p.add_argument("--warm", action="store_true", help="warm-up for large batch training")
    p.add_argument("--trial", type=str, default="0", help="id for recording multiple runs")
    p.add_argument("--sec", action="store_true", help="add sec loss")
    p.add_argument("--sec_wei", type=float, default=0.0)
    p.add_argument("--norm_momentum", type=float, default=1.0)
    p.add_argument("--l2reg", action="store_true", help="add l2reg loss")
    p.add_argument("--l2reg_wei", type=float, default=0.0)
    p.add_argument("--ckpt", type=str, default="", help="path to pre-trained model")
    p.add_argument("--local_rank", "--local-rank", dest="local_rank", type=int, default=0)
    p.add_argument("--ngpu", type=int, default=None,
                   help="world size (defaults to WORLD_SIZE from the launcher)")
    g = p.add_argument_group("pretraining additions")
    g.add_argument("--optimizer", type=str, default="sgd", choices=["sgd", "lars"])
    g.add_argument("--grad_semantics", type=str, default="ref", choices=["ref", "exact"],
                   help="ref: DDP-mean of the global loss gradient (reference, SURVEY Q2); exact: W x that")
    g.add_argument("--grad_compress", type=str, default="none", choices=["none", "bf16"],
                   help="gradient bucket all-reduce payload: fp32 (reference DDP) or bf16 (half the "
                        "xGMI bytes; sums rounded to bf16)")
    g.add_argument("--base_temperature", type=float, default=0.07)
    g.add_argument("--contrast_mode", type=str, default="all", choices=["all", "one"])
    g.add_argument("--resume", type=str, default="", help="resume model+optimizer+epoch+state from a ckpt")
    g.add_argument("--micro_batch", type=int, default=0,
                   help="gradient-cache micro-batching: encoder forward/backward in chunks of this many "
                        "VIEWS per rank (0 = whole local batch); the contrastive loss still sees the full batch")
    _add_common_new_flags(p)
    return p


def _finish_common(opt, prefix_dirs: bool):
    it = opt.lr_decay_epochs.split(",") if isinstance(opt.lr_decay_epochs, str) else opt.lr_decay_epochs
    opt.lr_decay_epochs = [int(x) for x in it if str(x).strip() != ""]
    return opt


def _warm_fields(opt):
    # main_supcon.py:120-131 / main_linear.py:79-89
    if opt.warm:
        opt.model_name = f"{opt.model_name}_warm"
        opt.warmup_from = 0.01
        opt.warm_epochs = 10
        if opt.cosine:
            eta_min = opt.learning_rate * (opt.lr_decay_rate ** 3)
            opt.warmup_to = eta_min + (opt.learning_rate - eta_min) * (
                1 + math.cos(math.pi * opt.warm_epochs / opt.epochs)) / 2
        else:
            opt.warmup_to = opt.learning_rate


def unique_dir(path: str) -> str:
    """Collision guard for minute-resolution run folders."""
    if not os.path.exists(path):
        return path
    i = 1
    while os.path.exists(f"{path}_{i}"):
        i += 1
    return f"{path}_{i}"


def parse_pretrain(argv: Optional[Sequence[str]] = None, make_dirs: bool = True,
                   now: Optional[datetime.datetime] = None):
    opt = pretrain_parser().parse_args(argv)
    if opt.dataset == "path":
        assert opt.data_folder is not None and opt.mean is not None and opt.std is not None
    rank, local_rank, world = env_rank_info(opt.local_rank)
    opt.rank, opt.local_rank = rank, local_rank
    if opt.ngpu is None:
        opt.ngpu = world
    opt.world_size = opt.ngpu
    if opt.data_folder is None:
        opt.data_folder = "./datasets/"
    opt.model_path = os.path.join(opt.work_dir, f"{opt.dataset}_models")
    opt.tb_path = os.path.join(opt.work_dir, f"{opt.dataset}_tensorboard")
    _finish_common(opt, True)
    # main_supcon.py:109-117
    opt.model_name = "{}_{}_{}_lr_{}_decay_{}_bsz_{}_temp_{}_trial_{}".format(
        opt.method, opt.dataset, opt.model, opt.learning_rate, opt.weight_decay,
        opt.batch_size, opt.temp, opt.trial)
    if opt.cosine:
        opt.model_name = f"{opt.model_name}_cosine"
    if opt.sec:
        opt.model_name = f"{opt.model_name}_sec"
    if opt.batch_size > 256:
        opt.warm = True
    _warm_fields(opt)
    now = now or datetime.datetime.now()
    conf_work_path = f"{opt.dataset}_" + now.strftime("%m%d_%H%M") + "_"
    opt.conf_work_path = conf_work_path
    opt.tb_folder = os.path.join(opt.tb_path, conf_work_path + opt.model_name)
    opt.save_folder = os.path.join(opt.model_path, conf_work_path + opt.model_name)
    if make_dirs and opt.rank == 0:
        if os.path.isdir(opt.save_folder) and not opt.resume:
            opt.save_folder = unique_dir(opt.save_folder)
            opt.tb_folder = unique_dir(opt.tb_folder)
        os.makedirs(opt.tb_folder, exist_ok=True)
        os.makedirs(opt.save_folder, exist_ok=True)
    if opt.dataset == "path":
        opt.mean_t, opt.std_t = parse_tuple(opt.mean), parse_tuple(opt.std)
    else:
        opt.mean_t, opt.std_t = DATASET_STATS[opt.dataset]
    opt.n_cls = N_CLASSES.get(opt.dataset, 0)
    opt.record_norm_mean = None  # main_supcon.py:150
    if opt.batch_size % opt.world_size != 0:
        raise ValueError(f"--batch_size {opt.batch_size} must be divisible by world size {opt.world_size}")
    opt.local_batch = opt.batch_size // opt.world_size
    return opt


def linear_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("argument for training")
    # main_linear.py:24-61
    p.add_argument("--print_freq", type=int, default=10, help="print frequency")
    p.add_argument("--save_freq", type=int, default=10, help="save frequency")
    p.add_argument("--batch_size", type=int, default=512, help="batch_size")
    p.add_argument("--num_workers", type=int, default=16, help="num of workers to use")
    p.add_argument("--epochs", type=int, default=100, help="number of training epochs")
    p.add_argument("--learning_rate", type=float, default=0.1, help="learning rate")
    p.add_argument("--lr_decay_epochs", type=str, default="60,75,90", help="where to decay lr")
    p.add_argument("--lr_decay_rate", type=float, default=0.2, help="decay rate for learning rate")
    p.add_argument("--weight_decay", type=float, default=0, help="weight decay")
    p.add_argument("--momentum", type=float, default=0.9, help="momentum")
    p.add_argument("--model", type=str, default="resnet50")
    p.add_argument("--dataset", type=str, default="cifar10", choices=["cifar10", "cifar100"])
    p.add_argument("--cosine", action="store_true", help="using cosine annealing")
    p.add_argument("--warm", action="store_true", help="warm-up for large batch training")
    p.add_argument("--ckpt", type=str, default="", help="path to pre-trained model")
    g = p.add_argument_group("linear-probe additions")
    g.add_argument("--data_folder", type=str, default="./datasets/")
    g.add_argument("--val_batch_size", type=int, default=256)
    g.add_argument("--local_rank", "--local-rank", dest="local_rank", type=int, default=0)
    _add_common_new_flags(p)
    return p


def parse_linear(argv: Optional[Sequence[str]] = None, make_dirs: bool = True,
                 now: Optional[datetime.datetime] = None):
    opt = linear_parser().parse_args(argv)
    rank, local_rank, world = env_rank_info(opt.local_rank)
    opt.rank, opt.local_rank, opt.world_size = rank, local_rank, world
    _finish_common(opt, True)
    opt.model_name = "{}_{}_lr_{}_decay_{}_bsz_{}".format(
        opt.dataset, opt.model, opt.learning_rate, opt.weight_decay, opt.batch_size)
    if opt.cosine:
        opt.model_name = f"{opt.model_name}_cosine"
    _warm_fields(opt)
    opt.n_cls = N_CLASSES[opt.dataset]
    now = now or datetime.datetime.now()
    conf_work_path = "classifier_" + now.strftime("%m%d_%H%M") + "_"
    opt.conf_work_path = conf_work_path
    opt.tb_path = os.path.join(opt.work_dir, f"{opt.dataset}_tensorboard")
    opt.tb_folder = os.path.join(opt.tb_path, conf_work_path + opt.model_name)
    opt.model_path = os.path.join(opt.work_dir, f"{opt.dataset}_models")
    opt.save_folder = os.path.join(opt.model_path, conf_work_path + opt.model_name)
    if make_dirs and opt.rank == 0:
        if os.path.isdir(opt.save_folder):
            opt.save_folder = unique_dir(opt.save_folder)
            opt.tb_folder = unique_dir(opt.tb_folder)
        os.makedirs(opt.tb_folder, exist_ok=True)
        os.makedirs(opt.save_folder, exist_ok=True)
    opt.mean_t, opt.std_t = DATASET_STATS[opt.dataset]
    return opt
