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
