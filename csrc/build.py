#!/usr/bin/env python3
"""In-tree build of the gfx950 extension ``simclr_pytorch_distributed_amd/_C.so``.

Design (no hipify, no setuptools CUDAExtension): the HIP kernels in ``csrc/kernels``
are plain HIP (no torch headers) compiled by ``hipcc --offload-arch=gfx950``; the
binding TUs in ``csrc/bindings`` include torch headers and are compiled host-only.
Objects are cached under ``build/obj`` keyed on source mtime, included-header mtimes
and the flag string, and compiled in parallel. The final shared object is written
inside the package so it travels to the GPU box with the repo snapshot.

Usage: ``python csrc/build.py [--force] [--jobs N] [--debug] [--checked]``

``--checked`` builds ``_C_checked.so`` with device-side bounds checks (``SDX_DCHECK``:
every implicit-GEMM operand gather, augmentation source pixel, pooling window) that trap
with a message on violation; load it with ``SDX_CHECKED=1``.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "simclr_pytorch_distributed_amd")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(PKG, "_C.so")
ARCH = os.environ.get("SDX_OFFLOAD_ARCH", "gfx950")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce
    return ce.include_paths(), ce.library_paths(), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def _headers_mtime():
    m = 0.0
    for d in (os.path.join(CSRC, "include"),):
        for f in os.listdir(d):
            m = max(m, os.path.getmtime(os.path.join(d, f)))
    return m


def _sources():
    kern = sorted(os.path.join(CSRC, "kernels", f) for f in os.listdir(os.path.join(CSRC, "kernels"))
                  if f.endswith(".hip"))
    bind = sorted(os.path.join(CSRC, "bindings", f) for f in os.listdir(os.path.join(CSRC, "bindings"))
                  if f.endswith(".cpp"))
    return kern, bind


def build(force: bool = False, jobs: int | None = None, debug: bool = False, verbose: bool = False,
          checked: bool = False, variant: str = "", defines: list | None = None, sanitize: bool = False) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    inc_torch, lib_torch, abi = _torch_paths()
    hipcc = _hipcc()
    py_inc = sysconfig.get_paths()["include"]
    opt = ["-O0", "-g"] if debug else ["-O3"]
    common = ["-std=c++17", "-fPIC", f"-I{os.path.join(CSRC, 'include')}", "-Wno-unused-result",
              "-Wno-deprecated-declarations"]
    # variant: an experiment build _C_<variant>.so with extra kernel defines (loaded with
    # SDX_EXT_VARIANT=<variant>), e.g. --variant fragpin --define SDX_FRAG_PIN=1
    # sanitize: _C_san.so, the host binding layer (csrc/bindings) built with AddressSanitizer
    # + UndefinedBehaviorSanitizer (GCC runtimes); the device kernels are unchanged (GPU ASan
    # is not available). Load it under the ASan-instrumented Python launcher of
    # build_asan_python() (the ASan runtime must come first) with SDX_EXT_VARIANT=san.
    if sanitize:
        variant = "san"
    name = "_C_checked" if checked else ("_C_" + variant if variant else "_C")
    out_so = os.path.join(PKG, name + ".so")
    kflags = [hipcc, "-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              "-ffp-contract=fast"] + opt + common + (["-DSDX_CHECKED=1"] if checked else []) + \
        [f"-D{d}" for d in (defines or [])]
    bflags = [os.environ.get("CXX", "g++"), "-O2", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              "-I/opt/rocm/include",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
              f"-DTORCH_EXTENSION_NAME={name}", f"-I{py_inc}"] + [f"-I{p}" for p in inc_torch] + common + \
        (SAN_FLAGS if sanitize else [])
    kern, bind = _sources()

    # objects are keyed on the flags and the CONTENT of the source and of every header (an
    # mtime test misses an edit made while that source was compiling)
    hdr_h = hashlib.sha1()
    hdir = os.path.join(CSRC, "include")
    for f in sorted(os.listdir(hdir)):
        with open(os.path.join(hdir, f), "rb") as fh:
            hdr_h.update(f.encode() + fh.read())
    hdr_digest = hdr_h.hexdigest()

    def job(src, flags):
        with open(src, "rb") as fh:
            src_digest = hashlib.sha1(fh.read()).hexdigest()
        key = hashlib.sha1((" ".join(flags) + src + src_digest + hdr_digest).encode()).hexdigest()[:12]
        obj = os.path.join(OBJ_DIR, os.path.basename(src) + f".{key}.o")
        if not force and os.path.exists(obj):
            return obj, False
        cmd = flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
        return obj, True

    # igemm.hip: MFMA accumulators in arch VGPRs. Its 4-wave 64x128 wave tiles (cfgs 7/8) hold
    # 128 fp32 accumulators per lane; with the default AGPR heuristics hipcc copied them through
    # a temporary around every MFMA (~600 v_accvgpr moves per kernel); the VGPR form needs 256
    # VGPRs + 20 AGPRs and no copies. Every other instantiation compiles to the same code.
    per_file = {"igemm.hip": ["-mllvm", "--amdgpu-mfma-vgpr-form"]}
    tasks = [(s, kflags + per_file.get(os.path.basename(s), [])) for s in kern] + [(s, bflags) for s in bind]
    n = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=n) as ex:
        results = list(ex.map(lambda t: job(*t), tasks))
    objs = [o for o, _ in results]
    rebuilt = any(r for _, r in results)
    # the object set the .so was linked from: a source reverted to content whose object is
    # still cached rebuilds nothing and leaves the .so newer than every object, so an mtime
    # test alone would keep the stale link
    stamp = out_so + ".objs"
    linked = open(stamp).read() if os.path.exists(stamp) else ""
    if (rebuilt or force or not os.path.exists(out_so) or linked != "\n".join(objs)
            or os.path.getmtime(out_so) < max(os.path.getmtime(o) for o in objs)):
        libs = []
        for p in lib_torch:
            libs += [f"-L{p}", f"-Wl,-rpath,{p}"]
        libs += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64"]  # RCCL symbols resolve from torch's own librccl.so (a dependency of libtorch_hip)
        if sanitize:
            libs += _gcc_san_libs()
        tmp = out_so + ".tmp"
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs + libs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out_so)
        with open(stamp, "w") as fh:
            fh.write("\n".join(objs))
    return out_so


SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g1"]


def _gcc_san_libs():
    libs = []
    for n in ("libasan.so", "libubsan.so"):
        p = subprocess.run(["gcc", f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
        libs += [p, f"-Wl,-rpath,{os.path.dirname(p)}"]
    return libs


ASAN_PY = os.path.join(ROOT, "build", "asan_python")


def build_asan_python(force: bool = False) -> str:
    """A Python interpreter executable linked with the GCC ASan/UBSan runtimes, so the
    sanitizer runtime is first in the process and ``_C_san.so`` can be imported (the host
    binding layer runs instrumented; torch and the device kernels are not)."""
    src = os.path.join(CSRC, "tools", "asan_python.cpp")
    if not force and os.path.exists(ASAN_PY) and os.path.getmtime(ASAN_PY) >= os.path.getmtime(src):
        return ASAN_PY
    os.makedirs(os.path.dirname(ASAN_PY), exist_ok=True)
    cfg = sysconfig.get_config_vars()
    cmd = ["g++", "-O1", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", f"-I{sysconfig.get_paths()['include']}",
           src, "-o", ASAN_PY, f"-L{cfg['LIBDIR']}", f"-lpython{cfg['VERSION']}", f"-Wl,-rpath,{cfg['LIBDIR']}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"asan_python build failed\n{r.stderr}")
    return ASAN_PY


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--checked", action="store_true", help="device bounds checks -> _C_checked.so")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--variant", default="", help="experiment build _C_<variant>.so (SDX_EXT_VARIANT)")
    ap.add_argument("--define", action="append", default=[], help="extra kernel define NAME=VALUE")
    ap.add_argument("--sanitize", action="store_true",
                    help="host bindings under ASan+UBSan -> _C_san.so (+ the build/asan_python launcher)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    out = build(force=a.force, jobs=a.jobs, debug=a.debug, verbose=a.verbose, checked=a.checked, variant=a.variant,
                defines=a.define, sanitize=a.sanitize)
    if a.sanitize:
        print(build_asan_python())
    print(out)


if __name__ == "__main__":
    sys.exit(main())
