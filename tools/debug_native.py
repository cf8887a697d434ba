"""Layer-by-layer comparison of the native executor against torch (fp32 and bf16 autocast)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from simclr_pytorch_distributed_amd.models import executor as ex
from simclr_pytorch_distributed_amd.models.resnet import SupConResNet
from simclr_pytorch_distributed_amd.ops.bn import bn_act
from simclr_pytorch_distributed_amd.ops.conv import conv2d_nhwc

dev = torch.device("cuda:0")
torch.manual_seed(0)
name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
model = SupConResNet(name).to(dev).to(memory_format=torch.channels_last)
ref = SupConResNet(name).to(dev).to(memory_format=torch.channels_last)
ref.load_state_dict(model.state_dict())
x = torch.randn(32, 3, 32, 32, device=dev)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-20)).item()


# ---- forward, block by block ----
enc, renc = model.encoder, ref.encoder
xn = ex.to_nhwc_input(x)
y, s = conv2d_nhwc(xn, enc.conv1.weight, 1, 1, True, cin_pad=5)
out = bn_act(y, s, enc.bn1, True, True, None)
r = torch.relu(renc.bn1(renc.conv1(x)))
print(f"stem          rel {rel(out.permute(0, 3, 1, 2), r):.3e}")
outs, routs = [out], [r]
for i, (b, rb) in enumerate(zip(enc.blocks(), renc.blocks())):
    out = ex._bottleneck(b, out, True, None) if hasattr(b, "conv3") else ex._basic(b, out, True, None)
    r = rb(r)
    outs.append(out)
    routs.append(r)
    print(f"block {i:2d}      rel {rel(out.permute(0, 3, 1, 2), r):.3e}")
feat = out.float().mean(dim=(1, 2))
rfeat = torch.flatten(renc.avgpool(r), 1)
print(f"feat          rel {rel(feat, rfeat):.3e}")

# ---- backward with a simple random projection loss ----
w = torch.randn_like(rfeat)
(feat * w).sum().backward()
(rfeat * w).sum().backward()
for (n, p), (_, q) in zip(enc.named_parameters(), renc.named_parameters()):
    if p.grad is None:
        print("no grad", n)
        continue
    e = rel(p.grad, q.grad)
    if e > 3e-2 or "conv1" in n and "layer" not in n:
        print(f"  grad {n:40s} rel {e:.3e}")
print("max grad rel", max(rel(p.grad, q.grad) for (_, p), (_, q) in zip(enc.named_parameters(),
                                                                          renc.named_parameters())))

# ---- torch bf16 autocast as the precision yardstick ----
ref2 = SupConResNet(name).to(dev).to(memory_format=torch.channels_last)
ref2.load_state_dict(model.state_dict())
with torch.autocast("cuda", dtype=torch.bfloat16):
    f2 = ref2.encoder(x).float()
print(f"torch-bf16 feat rel {rel(f2, rfeat):.3e}")
(f2 * w).sum().backward()
print("torch-bf16 max grad rel", max(rel(p.grad, q.grad) for (_, p), (_, q) in zip(ref2.encoder.named_parameters(),
                                                                                    renc.named_parameters())))
