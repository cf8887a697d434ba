"""bench.py driver contract on CPU: 2 ranks under torch.distributed.run (gloo), the torch
backend and a small model. Checks the single JSON line rank 0 prints (keys, whole-job
value, weak scaling of the global batch) — the same code path the 8-GPU scaling run takes,
minus the GPU kernels."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_json_contract(tmp_path):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--backend", "torch", "--model", "resnet18",
           "--per_gpu_batch", "4"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    c = d["config"]
    assert c["global_batch"] == 8 and c["per_gpu_batch"] == 4 and c["parallelism"] == "dp2+syncbn"
    # the timed run is a training run: first (warm-up) and last (timed) step losses are reported
    assert isinstance(c["first_loss_local"], float) and isinstance(c["last_loss_local"], float)
    assert c["loss_steps"] == 1 + 3 + 2
    # value = whole-job images/s = global batch x steps / time
    assert abs(d["value"] - 8 * 1e3 / d["ms_per_step"]) / d["value"] < 0.01


def test_bench_self_launches_ranks(tmp_path):
    """``python bench.py --gpus 2`` with no external launcher starts its own 2 ranks
    (torch.distributed.run as a child process) and relays rank 0's JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SDX_BENCH_CHILD")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--backend", "torch", "--model", "resnet18", "--per_gpu_batch", "4"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2+syncbn"
    assert d["config"]["global_batch"] == 8


def test_bench_global_batch_is_strong_scaling(tmp_path):
    """--global_batch fixes the total batch (README headline: BS 256 over 2 GPUs)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--backend", "torch", "--model", "resnet18",
           "--global_batch", "8", "--dataset", "cifar100"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["scaling"] == "strong"
    assert d["config"]["global_batch"] == 8 and d["config"]["per_gpu_batch"] == 4
    assert d["config"]["dataset_shape"] == "cifar100"
