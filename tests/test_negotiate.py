"""Lock-step set-up of the native SyncBN communicators, gloo on CPU.

``comm.negotiate`` runs a multi-step set-up whose steps contain collectives; the ranks
agree after every step. A failure injected on ONE rank must make every rank stop after
that same step, run its own cleanup, and report failure together — no rank may enter
the next step's collective alone (that would hang the test, bounded by the spawn join).
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, d, fail_rank, fail_step):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        from simclr_pytorch_distributed_amd.parallel import comm
        log = []

        def step(i):
            # even steps are local (allocate / map / init: may fail), odd steps open with a
            # collective (id broadcast, handle gather, self-check) and may fail after it —
            # the shape of the real set-ups in parallel/comm.py and parallel/xgmi.py
            def f():
                log.append(f"enter{i}")
                if i % 2 == 1:
                    t = torch.ones(1)
                    dist.all_reduce(t)
                    assert t.item() == world
                if rank == fail_rank and i == fail_step:
                    raise RuntimeError(f"injected failure in step {i}")
                log.append(f"done{i}")
            return f

        def cleanup():
            log.append("cleanup")

        ok, err = comm.negotiate([step(i) for i in range(4)], cleanup)
        with open(os.path.join(d, f"r{rank}.txt"), "w") as f:
            f.write(f"{int(ok)} {type(err).__name__ if err is not None else '-'} " + ",".join(log))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,fail_step", [(2, 1, 2), (4, 3, 0), (4, 0, 3), (8, 5, 1), (2, -1, -1)])
def test_negotiate_lockstep(world, fail_rank, fail_step):
    """One rank fails in a local step (0, 2) or after a step's collective (1, 3)."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_entry, args=(world, port, d, fail_rank, fail_step), nprocs=world, join=True)
        res = [open(os.path.join(d, f"r{r}.txt")).read().split(" ", 2) for r in range(world)]
    if fail_rank < 0:
        for ok, err, log in res:
            assert ok == "1" and err == "-" and "cleanup" not in log
        return
    for r, (ok, err, log) in enumerate(res):
        assert ok == "0", (r, log)
        assert log.endswith("cleanup"), (r, log)
        assert f"enter{fail_step + 1}" not in log, (r, log)     # nobody went on alone
        assert (err == "RuntimeError") == (r == fail_rank), (r, err)


def _fastest_entry(rank, world, port, d):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        from simclr_pytorch_distributed_amd.parallel import comm
        names = ["xgmi-fused", "rccl-native", "local-bn"]
        # every rank measures xgmi faster, except rank world-1 (timing skew: a slow peer);
        # local-bn is the fastest everywhere but not eligible (a timing baseline only)
        ms = [10.0 + 0.1 * rank, 11.0, 5.0]
        if rank == world - 1:
            ms[0] = 13.0
        best, red = comm.agree_fastest(names, ms, eligible=[0, 1])
        with open(os.path.join(d, f"f{rank}.txt"), "w") as f:
            f.write(best + " " + ",".join(f"{v:.3f}" for v in red))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_agree_fastest_transport_under_skew(world):
    """SyncBN transport choice (engine/pretrain.py autotune_syncbn): per-rank timings that
    disagree (one slow rank) still give ONE choice on every rank — the option whose slowest
    rank is fastest — and an ineligible baseline is never chosen."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fastest_entry, args=(world, port, d), nprocs=world, join=True)
        res = [open(os.path.join(d, f"f{r}.txt")).read().split(" ") for r in range(world)]
    assert {b for b, _ in res} == {"rccl-native"}
    assert len({t for _, t in res}) == 1      # the same reduced vector everywhere
    assert res[0][1].split(",")[0] == "13.000"


def test_agree_fastest_single_process():
    from simclr_pytorch_distributed_amd.parallel import comm
    best, red = comm.agree_fastest(["a", "b", "c"], [3.0, 2.0, 2.0])
    assert best == "b" and red == [3.0, 2.0, 2.0]
