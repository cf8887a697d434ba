import os, sys, collections
sys.path.insert(0, os.getcwd())
import torch
from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
from simclr_pytorch_distributed_amd.models.executor import ModelRunner, to_nhwc_input
from simclr_pytorch_distributed_amd.optim.flat import FlatParams
from simclr_pytorch_distributed_amd.ops import sinks
m = SupConResNet("resnet18").cuda().to(memory_format=torch.channels_last)
f = FlatParams(m)
r = ModelRunner(m, "native", master=f.flat)
name = {id(p): n for n, p in m.named_parameters()}
cnt = collections.Counter()
order = []
sinks.add_listener(lambda p: (cnt.update([name[id(p)]]), order.append(("sink", name[id(p)]))))
for n, p in m.named_parameters():
    def h(p, n=n):
        cnt.update([n])
        order.append(("hook", n))
    p.register_post_accumulate_grad_hook(h)
x = to_nhwc_input(torch.randn(8, 3, 32, 32, device="cuda"))
r.forward(x).sum().backward()
bad = {k: v for k, v in cnt.items() if v != 1}
missing = [n for n, _ in m.named_parameters() if n not in cnt]
print("double:", bad, "missing:", missing, "total", len(cnt))
print(order[-8:])
