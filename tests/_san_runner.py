"""Shared driver of the sanitizer tests: run a Python snippet under build/asan_python with
the ASan+UBSan build of the host binding layer (_C_san.so) and check the report."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_PY = os.path.join(ROOT, "build", "asan_python")
SAN_SO = os.path.join(ROOT, "simclr_pytorch_distributed_amd", "_C_san.so")


def available() -> bool:
    return os.path.exists(ASAN_PY) and os.path.exists(SAN_SO)


def run(code: str, timeout: float = 240.0):
    env = dict(os.environ, SDX_EXT_VARIANT="san", SDX_AUTOBUILD="0", PYTHONPATH=ROOT,
               # leaks: the interpreter and torch hold allocations to exit; shadow-gap
               # protection conflicts with the HIP runtime's address-space reservations
               ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([ASAN_PY, "-c", code], env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    report = p.stderr
    bad = [k for k in ("ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer") if k in report]
    return p.returncode, p.stdout, report, bad
