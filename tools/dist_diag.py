#!/usr/bin/env python3
"""Diagnose W=2 vs W=1 differences of one native training step (tests/dist_gpu_worker.py):
runs the worker at W=1 and W=2 (both processes on cuda:0, gloo process group) under the
given environment overrides and prints the parameter-update difference and the parameters
whose gradients differ most.

python tools/dist_diag.py MODEL SYNCBN_COMM "ENV1" "ENV2" [W2]
  ENV1 / ENV2: space-separated VAR=value overrides for the W=1 / second runs ("" = none);
  W2 = world size of the second run (default 2; 1 compares two single-rank runs, e.g. a
  summation-order perturbation such as SDX_STAT_FUSE=3: the chaos floor of the network)
"""
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def launch(world, out, model, syncbn_comm, extra):
    rdv = os.path.join(out, f"rdv_{world}")
    procs = []
    for r in range(world):
        env = dict(os.environ, SDX_TEST_SYNCBN_COMM=syncbn_comm, SDX_TEST_MODEL=model, RANK=str(r), LOCAL_RANK="0",
                   WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", SDX_INIT_METHOD="file://" + rdv, PYTHONPATH=ROOT,
                   OMP_NUM_THREADS="4")
        env.update(extra)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_gpu_worker.py"), out],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    for p in procs:
        _, err = p.communicate(timeout=300)
        if p.returncode != 0:
            raise SystemExit(err[-3000:])


def main():
    model, comm = sys.argv[1], sys.argv[2]
    env1 = dict(kv.split("=", 1) for kv in sys.argv[3].split()) if len(sys.argv) > 3 else {}
    env2 = dict(kv.split("=", 1) for kv in sys.argv[4].split()) if len(sys.argv) > 4 else {}
    w2 = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    with tempfile.TemporaryDirectory() as d1, tempfile.TemporaryDirectory() as d2:
        launch(1, d1, model, "", env1)
        launch(w2, d2, model, comm, env2)
        ref = torch.load(os.path.join(d1, f"{model}_w1_r0.pt"), weights_only=True)
        a = torch.load(os.path.join(d2, f"{model}_w{w2}_r0.pt"), weights_only=True)
    rel = float((ref["flat"] - a["flat"]).norm() / ref["flat"].norm())
    print(f"{model} W=1 vs W={w2} comm={comm or 'gloo'} env1={env1} env2={env2}: param-update rel {rel:.4g}, "
          f"loss w1 {ref['loss']:.5f}")
    rows = []
    for n, o, k in zip(a["names"], a["offsets"], a["numels"]):
        g1, g2 = ref["grad"][o:o + k].double(), a["grad"][o:o + k].double()
        rows.append((float((g2 - g1).norm() / (g1.norm() + 1e-12)), n, float(g1.norm())))
    rows.sort(reverse=True)
    for r, n, gn in rows[:12]:
        print(f"  {r:.4g}  {n}  |g| {gn:.4g}")
    print("  median rel", sorted(r for r, _, _ in rows)[len(rows) // 2])


if __name__ == "__main__":
    main()
