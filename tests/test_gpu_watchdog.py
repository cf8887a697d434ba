"""Failure detection on the native SyncBN communicators.

* watchdog drill: a W=2 emulated communicator with a 1 s timeout, whose collective's
  completion event waits behind a bounded 4 s GPU stall — the host watchdog must end the
  process with status 3 after ~1 s, naming the communicator, instead of waiting.
* stalled peer on the xGMI one-shot path: 2 ranks share cuda:0 (gloo process group,
  xGMI arena registered as the native executor's SyncBN handle); rank 1 stalls at step 1
  (fault injection), so rank 0's BN all-reduce kernel never sees its flag. The kernel
  gives up at the --comm_timeout deadline, flags the error word, and rank 0 exits with
  status 3 and one clear line instead of hanging or training on stale statistics.
"""
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRILL = r"""
import sys, time, torch
sys.path.insert(0, {root!r})
from simclr_pytorch_distributed_amd.ops import _ext
m = _ext.require()
h = m.emu_small_comm(2, 1.0)
x = torch.ones(8, dtype=torch.float64, device="cuda:0")
m.small_all_reduce_(h, x)
torch.cuda.synchronize()
assert float(x[0]) == 2.0
print("armed", flush=True)
time.sleep(0.3)                      # past the 200 us record throttle
m.small_comm_stall_(h, 4.0, x)
torch.cuda.synchronize()
print("NOT ABORTED", flush=True)
"""


def test_watchdog_ends_a_stalled_collective(gpu):
    t0 = time.time()
    p = subprocess.run([sys.executable, "-c", DRILL.format(root=ROOT)], capture_output=True, text=True, timeout=120)
    dt = time.time() - t0
    assert p.returncode == 3, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    assert "armed" in p.stdout and "NOT ABORTED" not in p.stdout
    assert "collective failure on the native SyncBN communicator" in p.stderr, p.stderr[-2000:]
    assert "did not complete within 1.0 s" in p.stderr


def test_xgmi_stalled_peer_exits_3(gpu, tmp_path):
    rdv = "file://" + str(tmp_path / "rdv")
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", SDX_INIT_METHOD=rdv, PYTHONPATH=ROOT, OMP_NUM_THREADS="4",
                   SDX_FAULT_INJECT="rank=1,step=1,mode=hang,seconds=90")
        cmd = [sys.executable, os.path.join(ROOT, "main_supcon.py"), "--model", "resnet18", "--batch_size", "16",
               "--synthetic", "--synthetic_size", "64", "--epochs", "1", "--print_freq", "1", "--backend", "native",
               "--dist_backend", "gloo", "--ngpu", "2", "--syncBN", "--syncbn_comm", "xgmi", "--comm_timeout", "8",
               "--work_dir", str(tmp_path / f"r{r}")]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        out, err = procs[0].communicate(timeout=100)
    except subprocess.TimeoutExpired:
        for q in procs:
            q.kill()
        pytest.fail("rank 0 hung although its peer stalled on the xGMI SyncBN path")
    finally:
        procs[1].kill()
        procs[1].communicate()
    assert procs[0].returncode == 3, (procs[0].returncode, err[-3000:])
    assert "native SyncBN communicator (xGMI)" in err, err[-3000:]
    assert "peer rank 1" in err, err[-3000:]
