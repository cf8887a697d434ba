"""Host-side sanitizers: the binding layer (csrc/bindings, the shape/stride/
pointer plumbing in front of every kernel launch) built with ASan + UBSan (_C_san.so,
csrc/build.py --sanitize) and imported under an ASan-linked interpreter. On the CPU box
every op's argument validation runs on wrong devices / dtypes / shapes — each call must
raise a clean error with no sanitizer report. (The GPU run of the same build:
tests/test_gpu_sanitize.py.)"""
import pytest

from _san_runner import available, run

pytestmark = pytest.mark.skipif(not available(), reason="sanitizer build absent (python csrc/build.py --sanitize)")

CODE = r"""
import torch
from simclr_pytorch_distributed_amd.ops import _ext
m = _ext.require()
assert m.__name__.endswith("_C_san"), m.__name__
bf = torch.bfloat16
x4 = torch.zeros(2, 4, 4, 8, dtype=bf)
f1 = torch.zeros(8)
calls = [
    lambda: m.conv_fwd(x4, x4, 1, 0, True),
    lambda: m.conv_dgrad(x4, x4, 4, 4, 1, 0),
    lambda: m.conv_wgrad(x4, x4, 1, 1, 1, 0),
    lambda: m.bn_apply(x4, f1, f1),
    lambda: m.bn_bwd_apply(x4, None, x4, torch.zeros(24)),
    lambda: m.bn_stats_finalize(torch.zeros(3, 2, 8), 10.0, None, None, 1e-5, 0.1, False, None, None),
    lambda: m.head_fwd(torch.zeros(4, 16), torch.zeros(8, 16, dtype=bf), torch.zeros(8)),
    lambda: m.head_bwd(torch.zeros(4, 8), torch.zeros(4, 16, dtype=bf), None, torch.zeros(16, 8, dtype=bf), None,
                       torch.zeros(8, 16), torch.zeros(8)),
    lambda: m.rownorm_fwd(torch.zeros(4, 300), 1e-12),
    lambda: m.supcon_fwd(torch.zeros(4, 128), torch.zeros(8, 128), torch.zeros(4, dtype=torch.int32),
                         torch.zeros(4, dtype=torch.int32), torch.zeros(8, dtype=torch.int32), 2.0, 1.0, 1.0),
    lambda: m.gpu_augment(torch.zeros(2, 8, 8, 3, dtype=torch.uint8), torch.zeros(2, dtype=torch.long), 8, 2, 0,
                          [0.5] * 3, [0.5] * 3, 0.2, 1.0, 0.75, 1.33, 0.8, 0.4, 0.4, 0.4, 0.1, 0.2, True, True),
    lambda: m.gpu_augment(torch.zeros(99, dtype=torch.uint8), torch.zeros(2, dtype=torch.long), 8, 2, 0,
                          [0.5] * 3, [0.5] * 3, 0.2, 1.0, 0.75, 1.33, 0.8, 0.4, 0.4, 0.4, 0.1, 0.2, True, True,
                          None, torch.zeros(2, dtype=torch.long), None),
    lambda: m.sgd_step(torch.zeros(8), torch.zeros(8), torch.zeros(8), torch.zeros(1), 0.9, 1e-4, 1.0, False),
    lambda: m.maxpool_fwd(x4, 3, 2, 1),
    lambda: m.gap_fwd(x4),
    lambda: m.wprep(torch.zeros(8), torch.zeros(8, dtype=bf), torch.zeros(1, 7, dtype=torch.long), 1),
    lambda: m.small_all_reduce_(12345, torch.zeros(4, dtype=torch.float64)),
    lambda: m.rccl_comm_init(torch.zeros(3, dtype=torch.uint8), 2, 0),
    lambda: m.block_bwd(x4, [], [], [], [], [], 1, True, False, 0),
]
n = 0
for i, c in enumerate(calls):
    try:
        c()
    except (RuntimeError, TypeError, ValueError) as e:
        n += 1
    else:
        raise SystemExit(f"call {i} did not raise")
print("validated", n)
"""


def test_binding_validation_under_asan_ubsan():
    rc, out, err, bad = run(CODE)
    assert not bad, err[-4000:]
    assert rc == 0, (rc, out[-2000:], err[-4000:])
    assert "validated 19" in out, out
