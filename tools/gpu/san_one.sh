#!/bin/bash
# One GPU test under the ASan+UBSan host build, verbose: bash tools/gpu/san_one.sh TEST_NODE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/san
python - "$1" <<'PY'
import os, subprocess, sys
sys.path.insert(0, "tests")
from _san_runner import ASAN_PY, ROOT, san_env
env = san_env()
env["AMD_LOG_LEVEL"] = "1"
cmd = [ASAN_PY, "-X", "faulthandler", "-m", "pytest", sys.argv[1], "-x", "-v", "-s", "-m", "gpu", "-p", "no:cacheprovider"]
p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
open("gpurun_out/san/one.txt", "w").write(f"rc {p.returncode}\n" + p.stdout + "\n---stderr---\n" + p.stderr)
print("rc", p.returncode)
PY
tail -60 gpurun_out/san/one.txt
