"""Failure detection / fault injection, 2 gloo ranks on CPU.

Rank 1 is killed by the fault-injection hook at global step 1; rank 0 must not hang: its
next collective fails, and the guarded entry point exits with status 3 after logging one
"collective failure" line that names the rank.
"""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_dead_peer_gives_clean_error(tmp_path):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SDX_FAULT_INJECT="rank=1,step=1,mode=exit", OMP_NUM_THREADS="2",
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", PYTHONPATH=ROOT)
        cmd = [sys.executable, os.path.join(ROOT, "main_supcon.py"), "--model", "resnet18", "--batch_size", "8",
               "--synthetic", "--synthetic_size", "64", "--epochs", "1", "--print_freq", "1", "--backend", "torch",
               "--dist_backend", "gloo", "--ngpu", "2", "--comm_timeout", "60", "--work_dir", str(tmp_path / f"r{r}")]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("a rank hung after its peer died")
        outs.append((p.returncode, out, err))
    assert outs[1][0] == 17, outs[1][2][-2000:]
    assert outs[0][0] == 3, outs[0][2][-3000:]
    assert "rank 0: collective failure" in outs[0][2]


def test_fault_spec_parsing(monkeypatch):
    from simclr_pytorch_distributed_amd.utils import faults
    monkeypatch.setenv("SDX_FAULT_INJECT", "rank=0,step=2,mode=raise")
    monkeypatch.setattr(faults, "_SPEC", None)
    faults.maybe_inject(0, 1)
    faults.maybe_inject(1, 2)
    with pytest.raises(faults.InjectedFault):
        faults.maybe_inject(0, 2)
    monkeypatch.setattr(faults, "_SPEC", None)


def test_collective_failure_classifier():
    from simclr_pytorch_distributed_amd.utils.faults import is_collective_failure
    assert is_collective_failure(RuntimeError("Connection closed by peer [127.0.0.1]:1234"))
    assert not is_collective_failure(ValueError("bad shape"))
