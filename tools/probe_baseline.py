"""GPU probe: MFMA selftest + stock-PyTorch (MIOpen) ResNet-50 SimCLR step timing."""
import time, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
import simclr_pytorch_distributed_amd._C as C

dev = torch.device("cuda:0")
print(torch.cuda.get_device_name(0), flush=True)
A = torch.randn(16, 32, device=dev).bfloat16(); B = torch.randn(32, 16, device=dev).bfloat16()
out = C.mfma16_selftest(A, B)
ref = A.float() @ B.float()
print("selftest max err", (out - ref).abs().max().item(), flush=True)

def run(bs, cl, dtype, steps=10, warm=5):
    torch.manual_seed(0)
    m = SupConResNet("resnet50").to(dev)
    if cl: m = m.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(bs, 3, 32, 32, device=dev)
    if cl: x = x.contiguous(memory_format=torch.channels_last)
    def step():
        with torch.autocast("cuda", dtype=dtype, enabled=dtype != torch.float32):
            f = m(x)
        f = F.normalize(f.float(), dim=1)
        s = f @ f.t() / 0.5
        s = s - torch.eye(bs, device=dev) * 1e9
        tgt = torch.arange(bs, device=dev).roll(bs // 2)
        loss = F.cross_entropy(s, tgt)
        opt.zero_grad(set_to_none=True); loss.backward(); opt.step()
        return loss
    for _ in range(warm): step()
    torch.cuda.synchronize(); t = time.time()
    for _ in range(steps): step()
    torch.cuda.synchronize(); dt = (time.time() - t) / steps
    print(f"views={bs} channels_last={cl} dtype={dtype}: {dt*1e3:.2f} ms/step  {bs/2/dt:.0f} src img/s", flush=True)

for cl in (True, False):
    for dt in (torch.bfloat16,):
        run(512, cl, dt)
run(512, True, torch.float32)
