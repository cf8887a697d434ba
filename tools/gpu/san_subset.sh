#!/bin/bash
# The sanitizer subset of the GPU tests, verbose (ASan+UBSan host build). -> gpurun_out/san/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/san
python - <<'PY'
import os, subprocess, sys
sys.path.insert(0, "tests")
from _san_runner import ASAN_PY, ROOT, san_env
FILES = ["tests/test_gpu_head.py", "tests/test_gpu_comm.py", "tests/test_gpu_bn.py", "tests/test_gpu_misc.py"]
cmd = [ASAN_PY, "-m", "pytest", *FILES, "-x", "-v", "-m", "gpu", "-p", "no:cacheprovider", "-k", "not fuzz and not checked"]
p = subprocess.run(cmd, env=san_env(), capture_output=True, text=True, timeout=600, cwd=ROOT)
open("gpurun_out/san/out.txt", "w").write(p.stdout + "\n---stderr---\n" + p.stderr)
print("rc", p.returncode)
PY
tail -40 gpurun_out/san/out.txt
