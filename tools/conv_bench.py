"""Per-shape convolution benchmark: native implicit-GEMM MFMA kernels vs MIOpen (torch
channels_last bf16) on the ResNet-50 CIFAR shapes at 512 views per GPU.

Usage: python tools/conv_bench.py [--views 512] [--iters 20] [--cfg -1]
Prints one line per (layer shape, pass) with µs and TFLOP/s, and the totals.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from simclr_pytorch_distributed_amd.ops import _ext


def resnet50_convs(n, hw=32):
    """(name, N, H, W, C, K, R, stride, pad, count) for every distinct conv of ResNet-50 (CIFAR stem)."""
    out = [("stem", n, hw, hw, 8, 64, 3, 1, 1, 1)]
    cin, h = 64, hw
    for li, (planes, blocks, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        for b in range(blocks):
            s = stride if b == 0 else 1
            ho = h // s
            tag = f"l{li + 1}.{'0' if b == 0 else 'x'}"
            cnt = 1 if b == 0 else blocks - 1
            if b == 0 or b == 1:
                out.append((tag + ".c1", n, h, h, cin, planes, 1, 1, 0, cnt))
                out.append((tag + ".c2", n, h, h, planes, planes, 3, s, 1, cnt))
                out.append((tag + ".c3", n, ho, ho, planes, planes * 4, 1, 1, 0, cnt))
                if b == 0:
                    out.append((tag + ".sc", n, h, h, cin, planes * 4, 1, s, 0, 1))
            cin, h = planes * 4, ho
    return out


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3   # µs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--no_miopen", action="store_true")
    a = ap.parse_args()
    m = _ext.require()
    dev = torch.device("cuda")
    tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
    print(f"{'shape':14s} {'pass':6s} {'M':>8s} {'N':>5s} {'K':>5s} {'native_us':>10s} {'TF/s':>7s} "
          f"{'miopen_us':>10s} {'TF/s':>7s}")
    for (name, N, H, W, C, K, R, st, pad, cnt) in resnet50_convs(a.views):
        x = torch.randn(N, H, W, C, device=dev).bfloat16()
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).bfloat16()
        P = (H + 2 * pad - R) // st + 1
        dy = torch.randn(N, P, P, K, device=dev).bfloat16()
        wt = w.permute(3, 1, 2, 0).contiguous()
        flops = 2.0 * N * P * P * K * R * R * C
        xc = x.permute(0, 3, 1, 2)          # NCHW view, channels_last memory
        wc = w.permute(0, 3, 1, 2)
        dyc = dy.permute(0, 3, 1, 2)
        runs = {
            "fwd": (lambda: m.conv_fwd(x, w, st, pad, True, a.cfg),
                    lambda: F.conv2d(xc, wc, stride=st, padding=pad)),
            "dgrad": (lambda: m.conv_dgrad(dy, wt, H, W, st, pad, a.cfg),
                      lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [st, st], [pad, pad], [1, 1],
                                                                  False, [0, 0], 1, [True, False, False])),
            "wgrad": (lambda: m.conv_wgrad(dy, x, R, R, st, pad, 0, a.cfg),
                      lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [st, st], [pad, pad], [1, 1],
                                                                  False, [0, 0], 1, [False, True, False])),
        }
        if R == 1 and st > 1:
            # what the step runs for a strided 1x1 shortcut (block_bwd sub_addend): the data
            # gradient lives on the stride-s subgrid only, so it is a stride-1 1x1 dgrad on the
            # P x Q grid that the block's final dgrad adds there (no zero sub-pixel classes)
            runs["dgrad_c"] = (lambda: m.conv_dgrad(dy, wt, P, P, 1, 0, a.cfg), runs["dgrad"][1])
        t_of = {}
        for ps, (nat, mio) in runs.items():
            if name == "stem" and ps == "dgrad":
                continue
            tn = timeit(nat, a.iters)
            tm = 0.0 if a.no_miopen or name == "stem" or ps == "dgrad_c" else timeit(mio, a.iters)
            if ps == "dgrad_c":
                # replaces the full-grid dgrad row in the totals
                tot["dgrad"][0] += (tn - t_of["dgrad"]) * cnt
                print(f"{name:14s} {ps:6s} {N * P * P:8d} {C:5d} {K:5d} {tn:10.1f} {flops / tn / 1e6:7.1f} "
                      f"{tm:10.1f} {flops / tm / 1e6 if tm else 0:7.1f}  x{cnt} (as run in the step)", flush=True)
                continue
            t_of[ps] = tn
            tot[ps][0] += tn * cnt
            tot[ps][1] += tm * cnt
            Mg = N * P * P if ps != "wgrad" else K
            print(f"{name:14s} {ps:6s} {Mg:8d} {K if ps == 'fwd' else C:5d} {R * R * (C if ps != 'dgrad' else K):5d} "
                  f"{tn:10.1f} {flops / tn / 1e6:7.1f} {tm:10.1f} {flops / tm / 1e6 if tm else 0:7.1f}  x{cnt}",
                  flush=True)
    for ps, (tn, tm) in tot.items():
        print(f"TOTAL {ps:6s} native {tn / 1e3:8.2f} ms   miopen {tm / 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
