"""Linear-probe evaluation engine — replaces main_linear.py:119-288 (+ main_ce.py:19-68 loaders).

Frozen encoder (eval-mode BN, no grad) + ``LinearClassifier`` trained with SGD and
cross-entropy; validation top-1/top-5 every epoch; the reported number is the best
validation top-1 (and the top-5 of that epoch), as in main_linear.py:284-288.

Fixes vs reference: checkpoint weights are always loaded (prefix-tolerant),
independent of GPU count. Augmentation runs on the GPU (RandomResizedCrop + flip +
normalize for training, normalize for validation) from the HBM-resident dataset.

Native backend (ops/linear_probe.py): the frozen encoder runs with every
eval-mode BatchNorm folded into its conv (one implicit-GEMM launch per conv + BN + ReLU, no
BN kernels), and the classifier's logits, cross-entropy, top-1/5 hits, gradient and SGD
update are two fused launches per batch; the meters stay on the device.
"""
from __future__ import annotations

import logging
import sys
import time
from typing import Optional

import torch
import torch.nn.functional as F

from ..data.augment import AugConfig, augment, nhwc8_to_nchw
from ..data.datasets import build_dataset
from ..data.sampler import DistributedIndexSampler
from ..models.executor import ModelRunner
from ..models.resnet import LinearClassifier, SupConResNet
from ..optim.schedules import adjust_learning_rate, warmup_learning_rate
from ..parallel import comm
from ..utils.logging import setup_logging
from ..utils.meters import AverageMeter, accuracy
from ..utils.profiling import PhaseTimer
from . import checkpoint as ckpt_mod
from .pretrain import resolve_backend, step_seed


class LinearEngine:
    def __init__(self, opt, device: Optional[torch.device] = None, model: Optional[torch.nn.Module] = None):
        self.opt = opt
        rank, local_rank, world, dev = comm.init_distributed(opt.dist_backend, getattr(opt, "comm_timeout", 600.0), device=device)
        self.device = dev
        setup_logging(opt.save_folder, rank)
        logging.info(f"create {opt.conf_work_path} ...")
        torch.manual_seed(opt.seed)
        self.backend = resolve_backend(opt.backend, dev, opt.stem)
        if model is None:
            model = SupConResNet(opt.model, opt.head, opt.feat_dim, opt.stem)
            if opt.ckpt:
                st = ckpt_mod.load_checkpoint(opt.ckpt)
                ckpt_mod.load_model_state(model, st["model"])
                logging.info(f"loaded encoder from {opt.ckpt}")
            else:
                logging.warning("no --ckpt given: probing a randomly initialised encoder")
        model = model.to(dev)
        if dev.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        model.eval()
        for p in model.parameters():
            p.requires_grad_(False)
        self.model = model
        self.runner = ModelRunner(model, self.backend, opt.precision)
        self.classifier = LinearClassifier(opt.model, opt.n_cls).to(dev)
        self.folded = None
        self.native_ce = None
        if self.backend == "native":
            from ..ops import linear_probe
            self.folded = linear_probe.FoldedEncoder(model.encoder)
            if linear_probe.supported(self.classifier):
                self.native_ce = linear_probe.NativeLinearCE(self.classifier, opt.momentum, opt.weight_decay)
        self.criterion = torch.nn.CrossEntropyLoss()
        self.optimizer = torch.optim.SGD(self.classifier.parameters(), lr=opt.learning_rate, momentum=opt.momentum,
                                         weight_decay=opt.weight_decay)
        nw = getattr(opt, "num_workers", 1)
        tr = build_dataset(opt.dataset, opt.data_folder, True, opt.synthetic, opt.synthetic_size, 32, opt.seed,
                           workers=nw)
        va = build_dataset(opt.dataset, opt.data_folder, False, opt.synthetic, opt.synthetic_size, 32, opt.seed,
                           workers=nw)
        self.tr_x, self.tr_y = torch.from_numpy(tr.images).to(dev), torch.from_numpy(tr.labels).to(dev)
        self.va_x, self.va_y = torch.from_numpy(va.images).to(dev), torch.from_numpy(va.labels).to(dev)
        # the reference DataLoader keeps the last partial batch (main_ce.py set_loader)
        self.sampler = DistributedIndexSampler(len(tr), opt.batch_size, 1, 0, seed=opt.seed, drop_last=False)
        self.aug_train = AugConfig.linear_train(32, opt.mean_t, opt.std_t)
        self.aug_val = AugConfig.evaluation(32, opt.mean_t, opt.std_t)
        from ..utils.tb import Logger
        self.logger = Logger(opt.tb_folder, flush_secs=2)
        self.prof = PhaseTimer(getattr(opt, "profile", False), dev)

    def _features(self, x):
        if self.backend == "torch":
            x = nhwc8_to_nchw(x)
        with torch.no_grad():
            if self.folded is not None:
                return self.folded(x)
            return self.runner.encode(x, training=False).float()

    def _classify(self, feats, labels, train: bool):
        """(logits, loss, acc1, acc5) of a batch — device tensors; train: + the SGD step."""
        bsz = labels.shape[0]
        if self.native_ce is not None:
            if train:
                out, st = self.native_ce.train_batch(feats, labels, self.optimizer.param_groups[0]["lr"])
            else:
                out, st = self.native_ce.eval_batch(feats, labels)
            return out, st[0] / bsz, st[1] * (100.0 / bsz), st[2] * (100.0 / bsz)
        output = self.classifier(feats.detach())
        loss = self.criterion(output, labels)
        acc1, acc5 = accuracy(output, labels, topk=(1, 5))
        if train:
            self.optimizer.zero_grad()
            loss.backward()
            self.optimizer.step()
        return output, loss.detach(), acc1[0], acc5[0]

    def train_epoch(self, epoch):
        opt = self.opt
        self.classifier.train()
        self.sampler.set_epoch(epoch)
        iters = len(self.sampler)
        if opt.max_steps:
            iters = min(iters, opt.max_steps)
        bt, dtm, losses, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter(), AverageMeter(), AverageMeter()
        # every batch counts in the epoch meters (reference main_linear.py:151-155): the sums
        # stay on the device and reach the host once per print window
        win = torch.zeros(4, dtype=torch.float64, device=self.device)   # Σloss·b, Σacc1·b, Σacc5·b, Σb
        end = time.time()
        for idx_i, idx in enumerate(self.sampler.batches(self.device)):
            if idx_i >= iters:
                break
            dtm.update(time.time() - end)
            ph = self.prof.phase
            with ph("augment"):
                x = augment(self.tr_x, idx, self.aug_train, step_seed(opt.seed, epoch, idx_i, 0))
                labels = self.tr_y[idx]
            bsz = labels.shape[0]
            warmup_learning_rate(opt, epoch, idx_i, iters, self.optimizer)
            with ph("encoder"):
                feats = self._features(x)
            with ph("classifier"):
                output, loss, acc1, acc5 = self._classify(feats, labels, True)
                win += torch.stack([loss.double() * bsz, acc1.double() * bsz, acc5.double() * bsz,
                                    torch.tensor(float(bsz), dtype=torch.float64, device=self.device)])
            bt.update(time.time() - end)
            if (idx_i + 1) % opt.print_freq == 0 or idx_i + 1 == iters:
                sl, s1, s5, nb = win.tolist()       # one host sync per print window
                win.zero_()
                losses.update(sl / nb, nb)
                losses.val = loss.item()
                top1.update(s1 / nb, nb)
                top1.val = acc1.item()
                top5.update(s5 / nb, nb)
                logging.info("Train: [{0}][{1}/{2}]\tBT {bt.val:.3f} ({bt.avg:.3f})\t"
                             "DT {dt.val:.3f} ({dt.avg:.3f})\tloss {loss.val:.3f} ({loss.avg:.3f})\t"
                             "Acc@1 {top1.val:.3f} ({top1.avg:.3f})".format(
                                 epoch, idx_i + 1, iters, bt=bt, dt=dtm, loss=losses, top1=top1))
                if self.prof.enabled:
                    logging.info("phases (ms/step): " + PhaseTimer.format(self.prof.summary()))
                sys.stdout.flush()
            end = time.time()
        return losses.avg, top1.avg, top5.avg

    @torch.no_grad()
    def validate(self):
        opt = self.opt
        self.classifier.eval()
        n = self.va_x.shape[0]
        losses, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter()
        vb = opt.val_batch_size
        for i, s in enumerate(range(0, n, vb)):
            idx = torch.arange(s, min(s + vb, n), device=self.device)
            x = augment(self.va_x, idx, self.aug_val, 0)
            labels = self.va_y[idx]
            output, loss, acc1, acc5 = self._classify(self._features(x), labels, False)
            bsz = labels.shape[0]
            losses.update(loss.item(), bsz)
            top1.update(acc1.item(), bsz)
            top5.update(acc5.item(), bsz)
            if i % opt.print_freq == 0:
                logging.info("Test: [{0}/{1}]\tLoss {loss.val:.4f} ({loss.avg:.4f})\t"
                             "Acc@1 {top1.val:.3f} ({top1.avg:.3f})".format(
                                 i, (n + vb - 1) // vb, loss=losses, top1=top1))
        logging.info(" * Acc@1 {top1.avg:.3f}, Acc@5 {top5.avg:.3f}".format(top1=top1, top5=top5))
        return losses.avg, top1.avg, top5.avg

    def run(self):
        opt = self.opt
        best_acc, best_acc5 = 0.0, 0.0
        for epoch in range(1, opt.epochs + 1):
            adjust_learning_rate(opt, self.optimizer, epoch)
            t1 = time.time()
            loss, acc, acc5 = self.train_epoch(epoch)
            logging.info("Train epoch {}, total time {:.2f}, accuracy:{:.2f}".format(epoch, time.time() - t1, acc))
            self.logger.log_value("classifier/train_loss", loss, epoch)
            self.logger.log_value("classifier/train_acc1", acc, epoch)
            self.logger.log_value("classifier/train_acc5", acc5, epoch)
            vloss, vacc, vacc5 = self.validate()
            self.logger.log_value("classifier/val_loss", vloss, epoch)
            self.logger.log_value("classifier/val_acc1", vacc, epoch)
            self.logger.log_value("classifier/val_acc5", vacc5, epoch)
            if vacc > best_acc:
                best_acc, best_acc5 = vacc, vacc5
        logging.info("best accuracy: {:.2f}, accuracy5: {:.2f}".format(best_acc, best_acc5))
        self.logger.close()
        return best_acc, best_acc5
