import os, sys
sys.path.insert(0, os.getcwd())
import torch
from simclr_pytorch_distributed_amd.ops import _ext
from tools.conv_bench import timeit
m = _ext.require()
dev = torch.device("cuda")
for (N, H, C, K) in [(1024, 56, 256, 512), (1024, 28, 512, 1024), (1024, 14, 1024, 2048), (512, 32, 256, 512)]:
    x = torch.randn(N, H, H, C, device=dev).bfloat16()
    P = H // 2
    dy = torch.randn(N, P, P, K, device=dev).bfloat16()
    out = torch.empty(K, 1, 1, C, device=dev, dtype=torch.float32)
    t_gen = timeit(lambda: m.conv_wgrad(dy, x, 1, 1, 2, 0, 0, -1, out), 10)
    def sub():
        xs = x[:, ::2, ::2, :].contiguous()
        return m.conv_wgrad(dy, xs, 1, 1, 1, 0, 0, -1, out)
    t_sub = timeit(sub, 10)
    t_copy = timeit(lambda: x[:, ::2, ::2, :].contiguous(), 10)
    fl = 2.0 * N * P * P * C * K
    print(f"N{N} H{H} C{C} K{K}: strided kernel {t_gen:8.1f} us ({fl/t_gen/1e6:6.1f} TF/s)   subsample+stride1 {t_sub:8.1f} us (copy alone {t_copy:7.1f})", flush=True)
