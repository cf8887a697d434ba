"""Tracing / phase-timer plumbing (CPU)."""
import torch

from simclr_pytorch_distributed_amd.utils import profiling


def test_phase_timer_cpu():
    t = profiling.PhaseTimer(True, torch.device("cpu"))
    for _ in range(3):
        with t.phase("a"):
            sum(range(1000))
        with t.phase("b"):
            pass
    s = t.summary()
    assert list(s) == ["a", "b"] and all(v >= 0 for v in s.values())
    assert t.summary() == {}            # reset after reading
    assert "a " in profiling.PhaseTimer.format(s)


def test_disabled_timer_is_noop():
    t = profiling.PhaseTimer(False, torch.device("cpu"))
    with t.phase("x"):
        pass
    assert t.summary() == {}


def test_roctx_calls_never_raise():
    profiling.range_push("r")
    profiling.mark("m")
    profiling.range_pop()
    with profiling.trace_range("t"):
        pass


def test_pretrain_step_with_profile(tmp_path):
    from simclr_pytorch_distributed_amd.config import parse_pretrain
    from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
    opt = parse_pretrain(["--model", "resnet18", "--batch_size", "8", "--synthetic", "--synthetic_size", "64",
                          "--epochs", "1", "--max_steps", "2", "--print_freq", "1", "--profile", "--backend", "torch",
                          "--work_dir", str(tmp_path)], make_dirs=True)
    eng = PretrainEngine(opt, device=torch.device("cpu"))
    eng.train_epoch(1)
    assert eng.prof.enabled


def test_rocprof_summary_counts_only_the_step_window(tmp_path):
    """tools/rocprof_summary.py: per-step tables sum only the kernels of
    the last N complete steps (boundaries = wprep_kernel starts); set-up kernels before the
    window (a copyBuffer, the first steps) and the unfinished step after the last boundary
    are left out. --all keeps the old whole-run / N behaviour."""
    import csv
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = [("__amd_rocclr_copyBuffer", 0, 50)]          # set-up, before any step
    t = 100
    for step in range(5):                                 # 5 steps of 3 kernels, 1000 ns each
        for name, dur in (("wprep_kernel", 10), ("igemm_kernel<0, 128>", 300), ("sgd_kernel", 90)):
            rows.append((name, t, t + dur))
            t += 200
        t += 400
    d = tmp_path / "trace"
    d.mkdir()
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "rocprof_summary.py"), str(d), "--steps", "3"],
                         capture_output=True, text=True, check=True).stdout
    assert "step window: the last 3 complete steps" in out
    assert "copyBuffer" not in out
    lines = {l.split()[-1]: l.split() for l in out.splitlines() if "ms/step" in l}
    assert float(lines["sgd_kernel"][2]) == 1.0 and float(lines["wprep_kernel"][2]) == 1.0   # calls/step
    # (10 + 300 + 90) ns per step
    assert "TOTAL kernel time per step: 0.000 ms" in out
