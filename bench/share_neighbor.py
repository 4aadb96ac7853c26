#!/usr/bin/env python3
"""Noisy neighbour on a shared MI355X: what the time slices' CU masks buy a latency-bound job.

    python bench/share_neighbor.py [--mnist-epochs 40] [--llama llama3-1b] [--out profiles/r02_shares/share_neighbor.json]

Two pods hold half of one GPU each (time slices, ``topology/shares.py``, placed through the whole
flow): the paper's MNIST CNN (latency-bound: small kernels, a hipGraph per step) and a Llama-3.2-1B
shaped training job (compute-bound: large GEMMs that fill every CU they can get).  MNIST's step time
is measured (1) alone on its share, (2) next to the Llama job with the CU masks Allocate hands out
(``HSA_CU_MASK``: disjoint halves of the CUs), and (3) next to it without masks (both jobs may use
every CU: the hardware interleaves their workgroups, the plain time-slicing other device plugins
offer).  The Llama job starts first and runs long enough that MNIST's whole timed loop overlaps its
steady state; its own throughput is reported too.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from share_mnist import _env, _finish, pod_envs  # noqa: E402


def _mnist(steps, env):
    cmd = [sys.executable, "-m", "gpu_topology_on_k8s_amd.models.train", "--model", "mnist-cnn", "--batch", "64",
           "--steps", str(steps), "--warmup", "20", "--gemm-tuning", "off"]
    return subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=REPO, env=env)


def _llama(model, steps, env):
    cmd = [sys.executable, "-m", "gpu_topology_on_k8s_amd.models.train", "--model", model, "--batch", "2", "--seq", "2048",
           "--steps", str(steps), "--warmup", "3", "--gemm-tuning", "off"]
    return subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=REPO, env=env)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--mnist-epochs", type=int, default=40)
    ap.add_argument("--llama", default="llama3-1b")
    ap.add_argument("--llama-steps", type=int, default=600)
    ap.add_argument("--lead-s", type=float, default=25.0, help="head start of the Llama job (start-up + warm-up)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    steps = a.mnist_epochs * 60000 // 64
    envs = pod_envs()
    unmasked = [{k: v for k, v in e.items() if k != "HSA_CU_MASK"} for e in envs]
    res = {"mnist_steps": steps, "pod_envs": envs}
    alone = _finish(_mnist(steps, _env(envs[0])))
    res["mnist_alone_on_share"] = {"ms_per_step": round(alone["ms_per_step"], 4), "images_per_s": round(alone["throughput"])}
    print(json.dumps(res), flush=True)
    for label, pair in (("with_cu_masks", envs), ("without_cu_masks", unmasked)):
        big = _llama(a.llama, a.llama_steps, _env(pair[1]))
        time.sleep(a.lead_s)
        small = _finish(_mnist(steps, _env(pair[0])))
        llama = _finish(big)
        res[label] = {"mnist_ms_per_step": round(small["ms_per_step"], 4), "mnist_images_per_s": round(small["throughput"]),
                      "mnist_slowdown_vs_alone": round(small["ms_per_step"] / alone["ms_per_step"], 3),
                      "llama_tokens_per_s": round(llama["throughput"]), "llama_ms_per_step": round(llama["ms_per_step"], 2),
                      "llama_mfu": llama.get("mfu")}
        print(json.dumps({label: res[label]}), flush=True)
    print(json.dumps({"summary": res}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
