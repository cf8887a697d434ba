"""The bounds-checked build (csrc/build.py --checked): the conv and
augmentation kernels run clean under their device-side checks on ragged / strided /
padded shapes (a violation traps the kernel and fails the subprocess)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import torch, torch.nn.functional as F
from simclr_pytorch_distributed_amd.ops import _ext
m = _ext.require()
assert m.__name__.endswith("_C_checked"), m.__name__
for (N, H, W, C, K, R, st, pad) in [(3, 9, 7, 64, 72, 3, 1, 1), (2, 8, 8, 64, 128, 3, 2, 1), (4, 5, 5, 256, 64, 1, 2, 0)]:
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
    for cfg in range(4):
        y, s = m.conv_fwd(x, w, st, pad, True, cfg)
        dy = torch.randn_like(y)
        m.conv_dgrad(dy, w.permute(3, 1, 2, 0).contiguous(), H, W, st, pad, cfg)
        m.conv_wgrad(dy, x, R, R, st, pad, 0, cfg)
data = torch.randint(0, 255, (50, 32, 32, 3), dtype=torch.uint8, device="cuda")
idx = torch.randint(0, 50, (64,), device="cuda")
from simclr_pytorch_distributed_amd.data.augment import AugConfig, gpu_augment
gpu_augment(data, idx, AugConfig.simclr(32, (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)), 7)
torch.cuda.synchronize()
print("CHECKED-OK")
"""


def test_checked_build_runs_clean(gpu):
    if not os.path.exists(os.path.join(ROOT, "simclr_pytorch_distributed_amd", "_C_checked.so")):
        pytest.skip("checked build not present (python csrc/build.py --checked)")
    env = dict(os.environ, SDX_CHECKED="1", SDX_AUTOBUILD="0", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "CHECKED-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
