"""Host-side sanitizers on the GPU: a subset of the GPU suite — native
training steps through the engine (block executor, head executor, weight cache, fused
optimizers), the emulated-SyncBN executor path and native gather, the BN and head kernels
— re-run with the host binding layer built under ASan + UBSan (_C_san.so) in the
ASan-linked interpreter. Device code is unchanged (GPU ASan is not available); every
pointer, shape and stride the bindings compute before a launch is checked by the host
sanitizers. Any sanitizer report fails the test."""
import subprocess

import pytest

from _san_runner import ASAN_PY, ROOT, available, san_env

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not available(), reason="sanitizer build absent")]

FILES = ["tests/test_gpu_head.py", "tests/test_gpu_comm.py", "tests/test_gpu_bn.py", "tests/test_gpu_misc.py"]


def test_gpu_suite_subset_under_asan_ubsan(gpu):
    env = san_env()
    cmd = [ASAN_PY, "-m", "pytest", *FILES, "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
           "-k", "not fuzz and not checked"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    out = p.stdout + p.stderr
    for k in ("ERROR: AddressSanitizer", "runtime error:"):
        assert k not in out, out[-6000:]
    assert p.returncode == 0, out[-6000:]
    import re
    m = re.search(r"(\d+) passed", p.stdout)
    print(p.stdout.strip().splitlines()[-1])
    # (conftest asserts in every test that the _C_san module was the one loaded)
    assert m and int(m.group(1)) >= 40, p.stdout[-800:]
