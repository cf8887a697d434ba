#!/usr/bin/env python3
"""Per-BN SyncBN cost on one GPU (reference: main_supcon.py:222-224, torch
SyncBatchNorm = one collective per BN in forward and one in backward, 53 + 53 per step).

For each ResNet-50 BN width C (slab rows = the conv-epilogue tiles of that layer at 128
images x 2 views per GPU) it times, with HIP events over back-to-back calls:

* local    — single process: column reduction + finalize in one launch (no SyncBN);
* 3-launch — the RCCL-path kernel sequence minus the collective itself: reduce launch,
             the EMU communicator's in-place x·W (stands in for ncclAllReduce's kernel),
             finalize launch;
* fused    — the fused xGMI exchange over W emulated ranks (XEMU communicator): every
             rank's reduction, the arena stores, the per-group flag round trip and the
             rank-ordered sum, all in ONE launch. The W virtual ranks share this GPU, so
             it also pays W x the reduction work of one rank (upper bound of the real
             per-rank cost, minus the xGMI link latency of the real peers).
* solo     — ONE rank's share of the fused exchange (SDX_SYNCBN_EMU_SOLO arena): only virtual
             rank 0 runs; it reduces its slab, stores into all W arenas, publishes all W flags,
             polls its own flag (the other ranks count as published) and sums the W slots — the
             per-rank kernel cost of a real W-GPU run minus the xGMI hop latency.

python tools/syncbn_latency.py [W[,W...]] [iters]     (default 2,4,8)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

# (C, slab rows): ResNet-50 CIFAR at 256 views per GPU, conv epilogue tiles of 128 rows (64 for layer 4)
SHAPES = [(64, 2048), (128, 2048), (256, 2048), (128, 512), (512, 512), (256, 128), (1024, 128), (512, 32),
          (2048, 64)]


def _time(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters   # µs per call


def main():
    Ws = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8").split(",")]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()
    dev = torch.device("cuda:0")
    summary = []
    for W in Ws:
        he = m.emu_small_comm(W)
        hx = m.xgmi_emu_small_comm(W)
        os.environ["SDX_SYNCBN_EMU_SOLO"] = "1"
        hs = m.xgmi_emu_small_comm(W)
        del os.environ["SDX_SYNCBN_EMU_SOLO"]
        print(f"per-BN SyncBN cost, W = {W} emulated ranks on one GPU, {iters} back-to-back calls (us per BN)")
        print(f"{'C':>6} {'rows':>6} | {'local':>8} {'3-launch':>9} {'fused':>8} {'solo':>8} | solo - local")
        tot = {"local": 0.0, "emu3": 0.0, "fused": 0.0, "solo": 0.0}
        for C, rows in SHAPES:
            slab = torch.randn(rows, 2, C, device=dev).abs_()
            g = torch.ones(C, device=dev)
            b = torch.zeros(C, device=dev)
            rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
            cnt = float(rows * 128)
            args = (g, b, 1e-5, 0.1, True, rm, rv)

            def local():
                m.bn_stats_finalize(slab, cnt, *args)

            def emu3():
                s_ = m.bn_stats_reduce(slab)
                m.small_all_reduce_(he, s_)
                m.bn_finalize(s_, cnt * W, *args)

            def fused():
                m.syncbn_exchange_sums(hx, slab)

            def solo():
                m.syncbn_exchange_sums(hs, slab)

            t = {k: _time(f, iters) for k, f in (("local", local), ("emu3", emu3), ("fused", fused), ("solo", solo))}
            ref = slab.double().sum(0) * W
            got = m.syncbn_exchange_sums(hx, slab)
            torch.cuda.synchronize()
            assert torch.allclose(got, ref, rtol=1e-12, atol=1e-9), "fused exchange mismatch"
            for k in tot:
                tot[k] += t[k]
            print(f"{C:>6} {rows:>6} | {t['local']:8.2f} {t['emu3']:9.2f} {t['fused']:8.2f} {t['solo']:8.2f} | "
                  f"{t['solo'] - t['local']:+7.2f}")
        n = len(SHAPES)
        print(f"{'mean':>13} | {tot['local'] / n:8.2f} {tot['emu3'] / n:9.2f} {tot['fused'] / n:8.2f} "
              f"{tot['solo'] / n:8.2f} | {(tot['solo'] - tot['local']) / n:+7.2f}")
        summary.append((W, tot["local"] / n, tot["emu3"] / n, tot["fused"] / n, tot["solo"] / n))
        for h in (he, hx, hs):
            m.small_comm_destroy(h)
    print("summary (mean us per BN): W local 3-launch fused solo")
    for r in summary:
        print("  %d %8.2f %8.2f %8.2f %8.2f" % r)


if __name__ == "__main__":
    main()
