"""GPU probe: native ResNet-50 SimCLR step — correctness vs torch fp32, then timing."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from simclr_pytorch_distributed_amd.losses.supcon import DistributedContrastiveLoss
from simclr_pytorch_distributed_amd.models.executor import ModelRunner, to_nhwc_input
from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
from simclr_pytorch_distributed_amd.ops import _ext

dev = torch.device("cuda:0")
m = _ext.require()


def build(seed=0):
    torch.manual_seed(seed)
    model = SupConResNet("resnet50").to(dev)
    model = model.to(memory_format=torch.channels_last)
    return model


def correctness():
    model = build()
    ref = build()
    ref.load_state_dict(model.state_dict())
    x = torch.randn(16, 3, 32, 32, device=dev)
    crit = DistributedContrastiveLoss("SimCLR", 0.5, backend="native")
    crit_ref = DistributedContrastiveLoss("SimCLR", 0.5, backend="torch")
    f = ModelRunner(model, "native").forward(to_nhwc_input(x))
    loss = crit(f)
    loss.backward()
    fr = ref(x)
    lr = crit_ref(fr)
    lr.backward()
    print(f"loss native {loss.item():.5f} torch-fp32 {lr.item():.5f}")
    print("feat rel err", ((f - fr).norm() / fr.norm()).item())
    for (n, p), (_, q) in list(zip(model.named_parameters(), ref.named_parameters()))[::20]:
        e = ((p.grad - q.grad).norm() / q.grad.norm().clamp_min(1e-12)).item()
        print(f"  grad {n:40s} rel {e:.3e}")
    for (n, b), (_, c) in list(zip(model.named_buffers(), ref.named_buffers()))[:3]:
        print(f"  buf {n} maxdiff {(b.float() - c.float()).abs().max().item():.3e}")


def timing(views=512, steps=10, warm=3):
    model = build()
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    runner = ModelRunner(model, "native")
    crit = DistributedContrastiveLoss("SimCLR", 0.5, backend="native")
    data = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, device=dev)
    mean, std = (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)

    def step(i):
        idx = torch.randint(0, 50000, (views // 2,), device=dev)
        x = m.gpu_augment(data, idx, 32, 2, 1234 + i, list(mean), list(std), 0.2, 1.0, 3 / 4, 4 / 3, 0.8, 0.4, 0.4,
                          0.4, 0.1, 0.2, True, True)
        f = runner.forward(x)
        loss = crit(f)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for i in range(warm):
        step(i)
    torch.cuda.synchronize()
    t = time.time()
    for i in range(steps):
        loss = step(i)
    torch.cuda.synchronize()
    dt = (time.time() - t) / steps
    print(f"native views={views}: {dt * 1e3:.2f} ms/step  {views / 2 / dt:.0f} src img/s  loss {loss.item():.4f}",
          flush=True)


if __name__ == "__main__":
    if "--time-only" not in sys.argv:
        correctness()
    timing(steps=int(os.environ.get("STEPS", "10")))
