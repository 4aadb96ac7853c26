#!/usr/bin/env python3
"""Gaia Exp. 6 workload under GPU sharing: two MNIST trainings on one MI355X, whole GPU in turn vs
two 0.5 shares at once.

    python bench/share_mnist.py [--epochs 10] [--batch 64] [--reps 3] [--out profiles/r02_shares/share_mnist.json]

The paper measures its placements with the official MNIST sample (p.7 Figs. 11-12: training time,
mean of 10 runs).  Its production gain comes from sharing GPUs between containers (abstract).  Here
both halves of that meet on one GPU: the node is advertised as 2 time slices per GPU
(``topology/shares.py``), two pods asking for half a GPU each go through the whole flow (extender
/filter /sort /bind, GetPreferredAllocation, Allocate), and each trains the paper's CNN
(``models/mnist.py``, HIP kernels, whole step in a hipGraph) for ``--epochs`` x 60k synthetic
images with the envs Allocate gave it (``HSA_CU_MASK``: its half of the CUs).  Baseline: the same
two jobs one after the other, each on the whole GPU (what whole-GPU allocation does with two jobs
and one free GPU).  Reported: each job's training time (its timed steps) and the makespan of the
pair (wall clock, process start to last exit).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
_STRIP = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "HSA_CU_MASK")


def _cmd(steps: int, batch: int):
    return [sys.executable, "-m", "gpu_topology_on_k8s_amd.models.train", "--model", "mnist-cnn", "--batch", str(batch),
            "--steps", str(steps), "--warmup", "20", "--gemm-tuning", "off"]


def _env(extra=None):
    e = {k: v for k, v in os.environ.items() if k not in _STRIP}
    e.update(extra or {})
    return e


def _finish(p):
    so, se = p.communicate(timeout=900)
    if p.returncode != 0:
        raise RuntimeError(se[-2000:])
    return json.loads([ln for ln in so.splitlines() if ln.startswith("{")][-1])


def pod_envs(slices: int = 2):
    from gpu_topology_on_k8s_amd.k8s import Contract
    from gpu_topology_on_k8s_amd.sim import SimCluster
    from gpu_topology_on_k8s_amd.topology.discovery import discover
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    t = discover("auto")
    t.node_name = "gpu-node"
    envs = []
    with SimCluster({"gpu-node": time_slice(t, slices)}) as c:
        for name in ("job-a", "job-b"):
            c.submit(name, slices // 2, slices=True, annotations={Contract().fraction_key: "0.5"})
            r = c.schedule_pending()[0]
            if r.error:
                raise RuntimeError(r.error)
            resp = c.nodes["gpu-node"].kubelet.responses[f"default/{name}"].container_responses[0]
            envs.append({k: v for k, v in resp.envs.items() if k.startswith(("GTK_", "HSA_"))})
    return envs


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    steps = a.epochs * 60000 // a.batch
    envs = pod_envs()
    rows = []
    for rep in range(a.reps):
        t0 = time.perf_counter()
        seq = [_finish(subprocess.Popen(_cmd(steps, a.batch), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                        cwd=REPO, env=_env())) for _ in range(2)]
        seq_wall = time.perf_counter() - t0
        t0 = time.perf_counter()
        procs = [subprocess.Popen(_cmd(steps, a.batch), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=REPO,
                                  env=_env(e)) for e in envs]
        par = [_finish(p) for p in procs]
        par_wall = time.perf_counter() - t0
        row = {"rep": rep,
               "whole_gpu_in_turn": {"train_s": [round(o["ms_per_step"] * steps / 1e3, 3) for o in seq], "makespan_s": round(seq_wall, 2)},
               "two_half_shares": {"train_s": [round(o["ms_per_step"] * steps / 1e3, 3) for o in par], "makespan_s": round(par_wall, 2),
                                   "hbm_cap": [o.get("hbm_cap_fraction") for o in par]}}
        print(json.dumps(row), flush=True)
        rows.append(row)

    def mean(path):
        return round(statistics.mean(path(r) for r in rows), 3)

    summary = {
        "epochs": a.epochs, "batch": a.batch, "steps_per_job": steps, "reps": a.reps, "pod_envs": envs,
        "whole_gpu_in_turn": {"train_s_per_job": mean(lambda r: statistics.mean(r["whole_gpu_in_turn"]["train_s"])),
                              "makespan_s": mean(lambda r: r["whole_gpu_in_turn"]["makespan_s"])},
        "two_half_shares": {"train_s_per_job": mean(lambda r: statistics.mean(r["two_half_shares"]["train_s"])),
                            "makespan_s": mean(lambda r: r["two_half_shares"]["makespan_s"])},
    }
    summary["makespan_ratio"] = round(summary["two_half_shares"]["makespan_s"] / summary["whole_gpu_in_turn"]["makespan_s"], 3)
    summary["gpu_time_ratio"] = round(summary["two_half_shares"]["train_s_per_job"] / (2 * summary["whole_gpu_in_turn"]["train_s_per_job"]), 3)
    print(json.dumps({"summary": summary}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"summary": summary, "runs": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
