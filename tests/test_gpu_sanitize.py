"""Host-side sanitizers on the GPU: a subset of the GPU suite — native
training steps through the engine (block executor, head executor, weight cache, fused
optimizers), the emulated-SyncBN executor path and native gather, the BN and head kernels
— re-run with the host binding layer built under ASan + UBSan (_C_san.so) in the
ASan-linked interpreter. Device code is unchanged (GPU ASan is not available); every
pointer, shape and stride the bindings compute before a launch is checked by the host
sanitizers. Any sanitizer report fails the test."""
import os
import subprocess

import pytest

from _san_runner import ASAN_PY, ROOT, available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not available(), reason="sanitizer build absent")]

FILES = ["tests/test_gpu_head.py", "tests/test_gpu_comm.py", "tests/test_gpu_bn.py", "tests/test_gpu_misc.py"]


def test_gpu_suite_subset_under_asan_ubsan(gpu):
    env = dict(os.environ, SDX_EXT_VARIANT="san", SDX_AUTOBUILD="0", PYTHONPATH=ROOT,
               ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    cmd = [ASAN_PY, "-m", "pytest", *FILES, "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
           "-k", "not fuzz and not checked"]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    out = p.stdout + p.stderr
    for k in ("ERROR: AddressSanitizer", "runtime error:"):
        assert k not in out, out[-6000:]
    assert p.returncode == 0, out[-6000:]
    assert " passed" in p.stdout, p.stdout[-500:]   # (conftest asserts the _C_san module was loaded)
