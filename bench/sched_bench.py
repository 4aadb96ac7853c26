#!/usr/bin/env python3
"""Gaia experiments 1-4 through the whole stack: placement tables + mean scheduling time.

    python bench/sched_bench.py [--reps 500] [--out profiles/sched/sched_bench.json]

Paper p.6-7: each request is submitted REPS times from a fixed node state (Fig. 7 tree: SOC ->
{PXB{GPU0 c2, GPU1 c2}, PIX{GPU2 c1, GPU3 c1}}) and the chosen GPU sets are tallied (Tables I-IV);
Fig. 10 reports the mean scheduling time (2.53-3.56 s with Gaia on k8s 1.9).  Here every repetition
is a real pass through the in-process cluster: mini-scheduler -> HTTP extender (filter, sort, bind)
-> apiserver annotations -> kubelet GetPreferredAllocation + Allocate over gRPC -> device plugin.
``sched_ms`` covers filter+sort+bind (the paper's scheduling time); ``admit_ms`` the kubelet side.
Exp. 2 (fractional 0.5/0.4/0.1 GPUs) runs twice: through the placement core's Fragment policy on
the Fig. 7 tree, and through the cluster as XCP partitions of one GPU (``<prefix>/gpu-fraction``
on a 4-GPU node exposing 10 partitions per GPU: 0.4 GPU = 4 partitions).
A second section times the exact policy on an 8x MI355X node (the case this framework targets), and
the sort fan-out over a 1024-node cluster with the polling cache and with the LIST+WATCH informer
(counting the LIST calls the steady state makes).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import random
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_topology_on_k8s_amd.k8s import PodAssignment  # noqa: E402
from gpu_topology_on_k8s_amd.placement import PlacementPolicy, gaia_schedule  # noqa: E402
from gpu_topology_on_k8s_amd.sim import SimCluster  # noqa: E402
from gpu_topology_on_k8s_amd.topology import fixtures as fx  # noqa: E402
from gpu_topology_on_k8s_amd.topology.model import GPUInfo, LinkType, Topology  # noqa: E402

PAPER_SCHED_S = {"exp1": (2.53, 2.66), "exp2": (None, 3.45), "exp3": (2.64, 3.02), "exp4": (2.58, 3.56)}  # (k8s, Gaia), Fig. 10


def fig7_topology() -> Topology:
    tr = fx.f4_tree()
    cost = np.array([[tr.pair_cost(i, j) for j in range(4)] for i in range(4)], float)
    return Topology(gpus=[GPUInfo(index=i, numa=[0, 0, 1, 1][i], model="P4") for i in range(4)],
                    link_type=np.full((4, 4), int(LinkType.PCIE)), hops=np.ones((4, 4), int), cost=cost, node_name="p4")


def run_exp(name: str, k: int, pre_used, reps: int, policy: str = "gaia", topo_fn=fig7_topology):
    tally = collections.Counter()
    sched, admit = [], []
    pol = PlacementPolicy(tie_break="random")
    with SimCluster({"node": topo_fn()}, policy_name=policy, policy=pol) as c:
        c.extender.cfg.seed = 0
        for i in range(reps):
            pods = []
            if pre_used:
                p = c.api.create_pod(__import__("gpu_topology_on_k8s_amd.k8s.objects", fromlist=["make_pod"]).make_pod(
                    f"busy{i}", gpus=len(pre_used), node="node", annotations=PodAssignment(list(pre_used), True, 1).to_annotations()))
                pods.append(("busy", p))
            c.submit(f"req{i}", k)
            (r,) = c.schedule_pending(admit=True)
            tally[tuple(r.allocated)] += 1
            sched.append(r.sched_ms)
            admit.append(r.admit_ms)
            c.delete(f"req{i}")
            if pre_used:
                c.api.delete_pod("default", f"busy{i}")
    return {
        "experiment": name, "request_gpus": k, "used_before": list(pre_used), "reps": reps, "policy": policy,
        "table": {",".join(f"gpu{g}" for g in s): n for s, n in sorted(tally.items())},
        "sched_ms_mean": statistics.mean(sched), "sched_ms_p50": statistics.median(sched),
        "sched_ms_p99": sorted(sched)[int(0.99 * (len(sched) - 1))], "admit_ms_mean": statistics.mean(admit),
        "paper_sched_s": PAPER_SCHED_S.get(name.split("-")[0]),
    }


def exp2_fragments(reps: int):
    tally = collections.Counter()
    for _ in range(reps):
        t = fx.f4_tree()
        t.mark_used([2], 0.5)
        a = gaia_schedule(t, 0.4, commit=True)
        b = gaia_schedule(t, 0.1, commit=True)
        tally[(tuple(a), tuple(b))] += 1
    return {"experiment": "exp2", "reps": reps, "table": {f"0.4->gpu{a[0]}, 0.1->gpu{b[0]}": n for (a, b), n in tally.items()},
            "note": "fractional GPUs have no k8s extended-resource form; placement core only (MI355X: XCP partitions)"}


def exp2_xcp_cluster(reps: int, node: str = "xcp"):
    """Gaia Table II through /filter, /sort, /bind, GetPreferredAllocation and Allocate: 0.5 of gpu2
    is held (5 of its 10 partitions), then a 0.4-GPU pod, then a 0.1-GPU pod.  ``node``: ``xcp`` = 10
    hardware partitions per GPU, ``slices`` = an SPX node whose device plugin advertises 10 time
    slices per GPU (topology/shares.py)."""
    from gpu_topology_on_k8s_amd.k8s import Contract
    from gpu_topology_on_k8s_amd.k8s.objects import make_pod
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    c0 = Contract()
    tally = collections.Counter()
    sched = []
    if node == "xcp":
        t = Topology.full_mesh(n=4, numa_split=1, partitions_per_gpu=10, node_name="p4")
    else:
        t = time_slice(Topology.full_mesh(n=4, numa_split=1, node_name="p4"), 10)
    with SimCluster({"p4": t}) as c:
        for i in range(reps):
            sl = node != "xcp"  # time slices are their own pool (amd.com/gpu-slice); XCPs are amd.com/gpu
            c.api.create_pod(make_pod(f"half{i}", gpus=5, node="p4", resource=c.nodes["p4"].resource,
                                      annotations=PodAssignment(list(range(20, 25)), True, 1).to_annotations()))
            c.submit(f"a{i}", 4, slices=sl, annotations={c0.fraction_key: "0.4"})
            (ra,) = c.schedule_pending()
            c.submit(f"b{i}", 1, slices=sl, annotations={c0.fraction_key: "0.1"})
            (rb,) = c.schedule_pending()
            gpu = lambda r: sorted({d // 10 for d in r.allocated})  # noqa: E731
            tally[(tuple(gpu(ra)), tuple(gpu(rb)))] += 1
            sched += [ra.sched_ms, rb.sched_ms]
            for n in (f"a{i}", f"b{i}"):
                c.delete(n)
            c.api.delete_pod("default", f"half{i}")
    return {"experiment": "exp2-xcp-cluster" if node == "xcp" else "exp2-timeslice-cluster", "reps": reps,
            "partitions_per_gpu" if node == "xcp" else "slices_per_gpu": 10,
            "table": {f"0.4->gpu{','.join(map(str, a))}, 0.1->gpu{','.join(map(str, b))}": n for (a, b), n in tally.items()},
            "sched_ms_mean": statistics.mean(sched), "paper_sched_s": PAPER_SCHED_S["exp2"]}


def scale_prioritize(n_nodes: int, pods: int = 20, k: int = 4, tm_policy: str = "none", split=None):
    """kube-scheduler's sort fan-out on a large cluster: one pending k-GPU pod x every node, repeated
    for `pods` same-size pods (no binds in between), extender called in process (no HTTP) so the
    numbers are the extender's own cost.  Decision cache off vs on (the LRU of scheduler.py).
    ``tm_policy``: every node's kubelet runs the Topology Manager with that policy (published by its
    plugin), so the extender replays the kubelet's NUMA alignment (placement/numa_align.py);
    ``split`` = (a, b): the pods have two containers of a and b GPUs."""
    import time

    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
    from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
    from gpu_topology_on_k8s_amd.placement.numa_align import TopologyManager, tm_labels

    api = FakeAPIServer()
    c = Contract()
    names = [f"node{i}" for i in range(n_nodes)]
    extra = tm_labels(TopologyManager(tm_policy, "container"), c.prefix) if tm_policy != "none" else {}
    for i, n in enumerate(names):
        t = fx.f7_mi355x(76.5, 0.03, i)
        api.create_node(make_node(n, labels={c.label_model: "MI355X", **extra}, annotations=encode_node_annotations(t, c),
                                  capacity={c.resource_name: "8"}))
    out = {"experiment": f"scale-prioritize-{n_nodes}-nodes" + (f"-tm-{tm_policy}" if tm_policy != "none" else ""),
           "nodes": n_nodes, "request_gpus": k, "pods": pods, "topology_manager": tm_policy, "containers": list(split or [k])}

    for mode, cache in (("cache_off", 0), ("cache_on", 4096), ("informer", 4096)):
        ext = TopologyExtender(api, ExtenderConfig(resync_s=60.0 if mode != "informer" else 0.0, decision_cache=cache))
        inf = None
        sync_ms = None
        if mode == "informer":
            t0 = time.perf_counter()
            inf = ext.cache.make_informer(watch_timeout=30.0)
            inf.start()
            inf.wait_synced(60)
            sync_ms = round((time.perf_counter() - t0) * 1e3, 2)
        ms = []
        lists_before = api.calls.get("list_pods", 0) + api.calls.get("list_nodes", 0)
        for i in range(pods):
            pod = api.create_pod(make_pod(f"p{mode}-{i}", gpus=0 if split else k, split=list(split) if split else None))
            t0 = time.perf_counter()
            ext.prioritize(pod, names)
            ms.append((time.perf_counter() - t0) * 1e3)
        lists = api.calls.get("list_pods", 0) + api.calls.get("list_nodes", 0) - lists_before
        out[mode] = {"first_ms": round(ms[0], 2), "steady_ms_mean": round(statistics.mean(ms[1:]), 2),
                     "steady_us_per_node": round(1e3 * statistics.mean(ms[1:]) / n_nodes, 2), "list_calls": lists}
        if sync_ms is not None:
            out[mode]["initial_sync_ms"] = sync_ms
            inf.stop()
    return out


def cpx_select(reps: int = 5):
    """The exact placement core on a CPX node (8 packages x 8 XCPs = 64 devices): median time per
    request size and used fraction, and whether the branch-and-bound finished exactly (symmetry
    breaking over interchangeable XCPs; before it, k = 16 took 364 ms and gave up exactness)."""
    import time

    from gpu_topology_on_k8s_amd.placement import select

    t = fx.f8_mi355x_cpx()
    rng = random.Random(7)
    rows = []
    for k in (1, 2, 4, 8, 16, 32):
        for frac in (0.0, 0.25, 0.5):
            ts, exact = [], True
            for _ in range(reps):
                used = rng.sample(range(64), int(64 * frac))
                if 64 - len(used) < k:
                    continue
                t0 = time.perf_counter()
                pl = select(t, k, used=used)
                ts.append((time.perf_counter() - t0) * 1e3)
                exact &= pl.exact
            if ts:
                rows.append({"k": k, "used_fraction": frac, "median_ms": round(statistics.median(ts), 3),
                             "max_ms": round(max(ts), 3), "exact": exact})
    return {"experiment": "cpx-64xcp-select", "reps": reps, "rows": rows}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--reps", type=int, default=500)
    ap.add_argument("--out", default="")
    ap.add_argument("--scale-nodes", type=int, default=1024, help="cluster size of the sort fan-out experiment (0: skip)")
    ap.add_argument("--scale-topology-manager", default="",
                    help="also run the fan-out with every kubelet's Topology Manager under this policy (single and 2+2 container pods)")
    ap.add_argument("--skip-tables", action="store_true", help="only the scale experiments")
    a = ap.parse_args()
    random.seed(0)
    results = [] if a.skip_tables else [
        run_exp("exp1-1gpu", 1, (), a.reps),
        run_exp("exp1-2gpu", 2, (), a.reps),
        exp2_fragments(a.reps),
        exp2_xcp_cluster(max(20, a.reps // 10)),
        exp2_xcp_cluster(max(20, a.reps // 10), node="slices"),
        run_exp("exp3", 1, (2,), a.reps),
        run_exp("exp4", 2, (2,), a.reps),
        run_exp("mi355x-exact-4gpu", 4, (), max(50, a.reps // 5), policy="exact", topo_fn=lambda: fx.f7_mi355x(76.5, 0.03, 1)),
        run_exp("mi355x-exact-1gpu-after-2", 1, (0, 1), max(50, a.reps // 5), policy="exact", topo_fn=lambda: fx.f7_mi355x(76.5, 0.03, 1)),
    ]
    if not a.skip_tables:
        results.append(cpx_select())
    if a.scale_nodes:
        results.append(scale_prioritize(a.scale_nodes))
        if a.scale_topology_manager:
            results.append(scale_prioritize(a.scale_nodes, tm_policy=a.scale_topology_manager))
            results.append(scale_prioritize(a.scale_nodes, tm_policy=a.scale_topology_manager, split=(2, 2)))
    for r in results:
        print(json.dumps(r))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
