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


def _setup_entry(rank, world, port, d, want, xgmi_fail, rccl_fail):
    """PretrainEngine._setup_syncbn_comm on a stub engine, with the native extension
    replaced by a fake whose xGMI arena creation / RCCL communicator join raise on ONE rank;
    comm.backend() reports nccl so the RCCL candidate is attempted (the uid broadcast runs
    on the gloo group itself)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    import datetime
    import types
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        from simclr_pytorch_distributed_amd.engine.pretrain import PretrainEngine
        from simclr_pytorch_distributed_amd.ops import _ext
        from simclr_pytorch_distributed_amd.parallel import comm
        log = []

        def xgmi_create(r, w, cap, t):
            if rank == xgmi_fail:
                raise RuntimeError("injected: arena allocation failed")
            log.append("xgmi_create")
            return 3

        def rccl_comm_init(uid, w, r, t):
            if rank == rccl_fail:
                raise RuntimeError("injected: ncclCommInitRank failed")
            log.append("rccl_init")
            return 7

        fake = types.SimpleNamespace(
            xgmi_create=xgmi_create, xgmi_handle=lambda i: torch.zeros(64, dtype=torch.uint8),
            xgmi_open=lambda i, h: (_ for _ in ()).throw(RuntimeError("no peer mapping on the CPU")),
            xgmi_destroy=lambda i: log.append(f"xgmi_destroy{i}"),
            small_comm_destroy=lambda h: log.append(f"comm_destroy{h}"),
            rccl_unique_id=lambda: torch.arange(128, dtype=torch.uint8),
            rccl_comm_init=rccl_comm_init,
            small_comm_abort=lambda h: log.append(f"abort{h}"))
        _ext.require = lambda: fake
        comm.backend = lambda: "nccl"
        torch.cuda.current_device = lambda: 0
        stub = types.SimpleNamespace(syncbn_transport="none")
        stub._activate_syncbn = lambda name: PretrainEngine._activate_syncbn(stub, name)
        opt = types.SimpleNamespace(syncbn_comm=want, comm_timeout=30.0)
        PretrainEngine._setup_syncbn_comm(stub, opt, torch.device("cuda"))
        with open(os.path.join(d, f"r{rank}.txt"), "w") as f:
            f.write(f"{stub.syncbn_transport} {','.join(stub._syncbn_cands) or '-'} {','.join(log) or '-'}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,want,xgmi_fail,rccl_fail,expect", [
    (2, "rccl", -1, 1, "none"),          # the RCCL join fails on rank 1: every rank falls back
    (4, "rccl", -1, 2, "none"),
    (2, "auto", 0, 1, "none"),           # both candidates fail, on different ranks
    # the xGMI arena fails on rank 3: every rank destroys its arena and joins RCCL together
    # (whose GPU self-check then fails everywhere alike: no GPU in this container)
    (4, "auto", 3, -1, "none"),
])
def test_syncbn_setup_falls_back_together(world, want, xgmi_fail, rccl_fail, expect):
    """a candidate transport whose creation raises on ONE rank during
    _setup_syncbn_comm leaves every rank with the same transport (no rank inside a
    collective alone: a hang would fail the spawn join), and a rank that had created its
    own handle before the failure aborts it."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_setup_entry, args=(world, port, d, want, xgmi_fail, rccl_fail), nprocs=world, join=True)
        res = [open(os.path.join(d, f"r{r}.txt")).read().split(" ") for r in range(world)]
    for r, (transport, cands, log) in enumerate(res):
        assert transport == expect, (r, transport, cands, log)
        if expect == "none":
            assert cands == "-", (r, cands)
            if want == "rccl" or rccl_fail >= 0:
                # the ranks that joined aborted their handle; the failing rank never had one
                assert ("abort7" in log) == (r != rccl_fail), (r, log)
        if xgmi_fail >= 0 and r != xgmi_fail:
            assert "xgmi_destroy3" in log, (r, log)   # arena created, then destroyed together
        if rccl_fail < 0:
            assert log.count("rccl_init") == 1 and log.endswith("abort7"), (r, log)
