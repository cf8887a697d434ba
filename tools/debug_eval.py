"""Pretrain a few steps (native), then check eval-mode features (native and torch) for
non-finite values and print BN running-stat ranges."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import logging
    logging.disable(logging.INFO)
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.data.augment import AugConfig, augment, nhwc8_to_nchw
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    from simclr_pytorch_distributed_amd.models.executor import ModelRunner
    opt = parse_pretrain(["--batch_size", "256", "--learning_rate", "0.5", "--temp", "0.5", "--cosine", "--synthetic",
                          "--synthetic_size", "4096", "--epochs", "1", "--seed", "1", "--backend", "native",
                          "--work_dir", "/tmp/dbg_eval"], make_dirs=False)
    eng = PretrainEngine(opt)
    eng.model.train()
    eng.sampler.set_epoch(1)
    for i, idx in enumerate(eng.sampler.batches(eng.device)):
        eng.train_step(idx, 1, i, 16)
        if i == 15:
            break
    torch.cuda.synchronize()
    bad = []
    for n, b in eng.model.named_buffers():
        if b.dtype.is_floating_point and not torch.isfinite(b).all():
            bad.append(n)
    print("non-finite buffers:", bad[:10])
    for n, mod in eng.model.named_modules():
        if isinstance(mod, torch.nn.BatchNorm2d) and n in ("encoder.bn1", "encoder.layer1.0.bn1", "encoder.layer4.2.bn3"):
            print(n, "rm", float(mod.running_mean.abs().max()), "rv", float(mod.running_var.min()),
                  float(mod.running_var.max()), "nbt", int(mod.num_batches_tracked))
    eng.model.eval()
    idx = torch.arange(256, device=eng.device)
    cfg = AugConfig.evaluation(32, opt.mean_t, opt.std_t)
    x = augment(eng.data, idx, cfg, 0)
    with torch.no_grad():
        fn = ModelRunner(eng.model, "native").encode(x, training=False).float()
        ft = ModelRunner(eng.model, "torch", "fp32").encode(nhwc8_to_nchw(x).float(), training=False).float()
    print("native eval feats finite:", bool(torch.isfinite(fn).all()), "max", float(fn.abs().max()))
    print("torch  eval feats finite:", bool(torch.isfinite(ft).all()), "max", float(ft.abs().max()))
    print("rel diff", float((fn - ft).norm() / ft.norm()))


if __name__ == "__main__":
    main()
