#!/usr/bin/env python3
"""Gaia B6 measured: does binding a GPU job's host threads to the GPU's own NUMA node pay on MI355X?

Paper p.3 §III.A binds every GPU to its nearest CPU cores so GPU<->CPU traffic does not cross
sockets (``gaia_gpu_topology_scheduler.md:45-46``).  The framework applies that binding in the
workload (``topology/cpus.py`` :func:`bind_workload`, ``GTK_CPUSET`` from Allocate).  This script
measures what it is worth on one GPU of the box, in child processes pinned three ways before they
import torch (first-touch puts their host buffers on the same NUMA node):

    local     --ncpus CPUs of the GPU's NUMA node (what bind_workload picks)
    remote    --ncpus CPUs of another NUMA node (the binding a topology-blind scheduler may give)
    unbound   every CPU the container allows (the kernel's choice)

Per child: pinned host->device and device->host copy GB/s (256 MiB, HIP events), pageable H2D GB/s
(the runtime stages through a pinned buffer with a CPU memcpy), the time to allocate and register
1 GiB of pinned memory, and two launch-bound training steps whose time is mostly host-side work:
the tiny Llama (``models.train --model tiny``) and the eager MNIST CNN (paper Exp. 6 workload).

    python bench/cpu_binding.py --reps 3 --ncpus 16 --out profiles/r03_cpubind/cpubind.json

The parent never initialises the GPU: it asks a child for the GPU's PCI address and reads NUMA
placement from sysfs.
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


def _read(path: str) -> str:
    with open(path) as f:
        return f.read().strip()


def child(cpus: str, workload: str = "micro") -> dict:
    """Runs in the pinned child: affinity first, then torch."""
    from gpu_topology_on_k8s_amd.topology.cpus import format_cpulist, parse_cpulist

    if cpus:
        s = parse_cpulist(cpus)
        os.sched_setaffinity(0, s)
        os.environ["OMP_NUM_THREADS"] = str(len(s))
    import torch

    from gpu_topology_on_k8s_amd.models.train import train

    torch.cuda.set_device(0)
    nb = 256 << 20
    out = {"cpus": format_cpulist(os.sched_getaffinity(0)), "n_cpus": len(os.sched_getaffinity(0))}
    if workload == "llama8b":  # the flagship step: GPU-bound, so binding should cost nothing here
        r = train("llama3-8b", batch=2, seq=4096, steps=4, warmup=2, placement="best", log=False, cpu_bind="off")
        out["llama8b_ms_per_step"] = round(r["ms_per_step"], 2)
        out["llama8b_tokens_per_s"] = round(r.get("tokens_per_s", 2 * 4096 / (r["ms_per_step"] / 1e3)), 1)
        return out

    def copy_gbps(src, dst, iters):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            dst.copy_(src, non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        return nb * iters / (e0.elapsed_time(e1) / 1e3) / 1e9

    t0 = time.perf_counter()
    big = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
    out["pin_alloc_1g_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    del big
    h = torch.ones(nb, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nb, dtype=torch.uint8, device="cuda")
    out["pinned_h2d_gbps"] = round(copy_gbps(h, d, 20), 2)
    out["pinned_d2h_gbps"] = round(copy_gbps(d, h, 20), 2)
    pg = torch.ones(nb, dtype=torch.uint8)
    t0 = time.perf_counter()
    for _ in range(5):
        d.copy_(pg)
    torch.cuda.synchronize()
    out["pageable_h2d_gbps"] = round(nb * 5 / (time.perf_counter() - t0) / 1e9, 2)
    del h, d, pg
    r = train("tiny", batch=1, seq=128, steps=40, warmup=5, placement="best", log=False, gemm_tuning="off", cpu_bind="off")
    out["llama_tiny_ms_per_step"] = round(r["ms_per_step"], 3)
    r = train("mnist-cnn", batch=64, steps=200, warmup=20, placement="best", log=False, gemm_tuning="off", graph="off",
              cpu_bind="off")
    out["mnist_eager_ms_per_step"] = round(r["ms_per_step"], 4)
    return out


def gpu_pci() -> str:
    p = subprocess.run([sys.executable, "-c", "from gpu_topology_on_k8s_amd.topology.identity import hip_device_bdfs;"
                        "print(hip_device_bdfs()[0])"], capture_output=True, text=True, timeout=300, cwd=REPO)
    if p.returncode != 0:
        raise RuntimeError(p.stderr[-1000:])
    return p.stdout.strip().splitlines()[-1]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--workload", default="micro", choices=["micro", "llama8b"],
                    help="micro: copies + launch-bound steps; llama8b: the Llama-3-8B training step (local/remote only)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ncpus", type=int, default=16, help="CPUs per pinned configuration (the box's CPU share)")
    ap.add_argument("--out", default="")
    ap.add_argument("--timeout", type=float, default=240.0, help="seconds per child")
    a = ap.parse_args()
    if a.child is not None:
        print(json.dumps(child(a.child, a.workload)), flush=True)
        return 0

    from gpu_topology_on_k8s_amd.topology.cpus import format_cpulist, parse_cpulist

    bdf = gpu_pci()
    dev = f"/sys/bus/pci/devices/{bdf.lower()}"
    gpu_numa = int(_read(f"{dev}/numa_node"))
    local_list = parse_cpulist(_read(f"{dev}/local_cpulist"))
    nodes = {}
    base = "/sys/devices/system/node"
    for e in sorted(os.listdir(base)):
        if e.startswith("node") and e[4:].isdigit():
            nodes[int(e[4:])] = parse_cpulist(_read(f"{base}/{e}/cpulist"))
    allowed = set(os.sched_getaffinity(0))
    local = sorted(allowed & (nodes.get(gpu_numa) or local_list))[: a.ncpus]
    remote_node = next((n for n in sorted(nodes) if n != gpu_numa and allowed & nodes[n]), None)
    remote = sorted(allowed & nodes[remote_node])[: a.ncpus] if remote_node is not None else []
    configs = {"local": format_cpulist(local), "remote": format_cpulist(remote), "unbound": ""}
    configs = {k: v for k, v in configs.items() if k == "unbound" or v}
    if a.workload == "llama8b":
        configs.pop("unbound", None)
    meta = {"gpu_bdf": bdf, "gpu_numa": gpu_numa, "gpu_local_cpulist": format_cpulist(local_list),
            "numa_nodes": {n: format_cpulist(c) for n, c in nodes.items()}, "allowed": format_cpulist(allowed),
            "remote_numa": remote_node, "configs": configs, "reps": a.reps, "workload": a.workload}
    print(json.dumps({"meta": meta}), flush=True)
    runs = {k: [] for k in configs}
    for rep in range(a.reps):
        order = list(configs) if rep % 2 == 0 else list(reversed(list(configs)))  # interleaved: no drift bias
        for name in order:
            print(json.dumps({"rep": rep, "config": name, "starting": True}), flush=True)
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", configs[name], "--workload", a.workload],
                               capture_output=True, text=True, timeout=a.timeout, cwd=REPO)
            if p.returncode != 0:
                print(f"child {name} failed: {p.stderr[-1500:]}", file=sys.stderr)
                return 1
            r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
            runs[name].append(r)
            print(json.dumps({"rep": rep, "config": name, **r}), flush=True)
    keys = ["pinned_h2d_gbps", "pinned_d2h_gbps", "pageable_h2d_gbps", "pin_alloc_1g_ms", "llama_tiny_ms_per_step",
            "mnist_eager_ms_per_step"] if a.workload == "micro" else ["llama8b_ms_per_step", "llama8b_tokens_per_s"]
    summary = {name: {k: round(statistics.median(r[k] for r in rs), 4) for k in keys} for name, rs in runs.items()}
    if "local" in summary and "remote" in summary:
        summary["remote_vs_local"] = {k: round(summary["remote"][k] / summary["local"][k], 4) for k in keys}
    doc = {"meta": meta, "median": summary, "runs": runs}
    print(json.dumps({"median": summary}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
