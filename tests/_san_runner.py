"""Shared driver of the sanitizer tests: run a Python snippet under build/asan_python with
the ASan+UBSan build of the host binding layer (_C_san.so) and check the report."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_PY = os.path.join(ROOT, "build", "asan_python")
SAN_SO = os.path.join(ROOT, "simclr_pytorch_distributed_amd", "_C_san.so")


def torch_lib() -> str:
    import importlib.util
    return os.path.join(os.path.dirname(importlib.util.find_spec("torch").origin), "lib")


def san_env() -> dict:
    """Environment of the ASan interpreter: the variant build, and torch/lib on the
    library path (the ASan dlopen interceptor resolves torch's runtime-loaded libraries,
    e.g. libcaffe2_nvrtc.so, without the caller's $ORIGIN run path)."""
    lib = torch_lib()
    return dict(os.environ, SDX_EXT_VARIANT="san", SDX_AUTOBUILD="0", PYTHONPATH=ROOT,
                LD_LIBRARY_PATH=lib + (":" + os.environ["LD_LIBRARY_PATH"] if os.environ.get("LD_LIBRARY_PATH") else ""),
                # leaks: the interpreter and torch hold allocations to exit; shadow-gap
                # protection conflicts with the HIP runtime's address-space reservations
                ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:halt_on_error=1",
                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def available() -> bool:
    return os.path.exists(ASAN_PY) and os.path.exists(SAN_SO)


def run(code: str, timeout: float = 240.0):
    p = subprocess.run([ASAN_PY, "-c", code], env=san_env(), capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    report = p.stderr
    bad = [k for k in ("ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer") if k in report]
    return p.returncode, p.stdout, report, bad
