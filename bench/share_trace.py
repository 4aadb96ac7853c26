#!/usr/bin/env python3
"""Cluster-level effect of GPU sharing (Gaia's fractional requests) on an MI355X cluster.

    python bench/share_trace.py [--nodes 16] [--jobs 4000] [--load 0.9] [--slices 4] [--out profiles/sched/share_trace.json]

Reference: the Gaia paper attributes its production gain ("GPU utilization improved by about 10%",
abstract and p.7 §V) to sharing GPUs between containers with fractional requests,
placed by its Fragment algorithm (paper p.4-5 Alg. 2: the GPU whose remaining share fits the request
most tightly).  This simulation replays one job trace that contains fractional jobs (notebooks,
inference, small experiments) against three ways a cluster can serve them, with the real placement
code for every decision:

    whole            no sharing: a 0.25-GPU job holds a whole GPU (the kubelet's integer resources)
    shares-bestfit   time-sliced nodes (device plugin ``--time-slices S``): the job takes ceil(m*S)
                     slices of one GPU chosen by ``placement.place_fraction`` (Fragment best fit,
                     partly used GPUs first) — what the extender does
    shares-firstfit  the same slices on the first GPU with room, nodes in order (Fragment without
                     best fit; also what the kubelet's lowest-free-ids choice amounts to)
    shares-spread    kube-scheduler's default LeastAllocated node (most free slices), then the first
                     GPU with room on it: fractions spread over every node

Whole-GPU jobs (1/2/4/8) are placed by the exact placement core on the GPUs no slice of which is in
use, node chosen by objective + node packing — identical in all three.  A fractional job runs its
base time on its share (its CUs are its own: ``HSA_CU_MASK``, measured on MI355X in
``profiles/r02_cumask``).  Metrics: goodput (work / GPU-time over the makespan), mean job completion
time, mean queueing delay (all jobs, fractional jobs, 8-GPU jobs).
"""
from __future__ import annotations

import argparse
import heapq
import json
import math
import os
import random
import statistics
import sys
from typing import Dict, List, Optional, Tuple


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_topology_on_k8s_amd.placement import NoFeasiblePlacement, PlacementPolicy, place_fraction, select  # noqa: E402
from gpu_topology_on_k8s_amd.placement.core import node_packing_term  # noqa: E402
from gpu_topology_on_k8s_amd.topology.model import Topology  # noqa: E402
from gpu_topology_on_k8s_amd.topology.shares import time_slice  # noqa: E402

POLICIES = ("whole", "shares-bestfit", "shares-firstfit", "shares-spread")
SIZES = (0.25, 0.5, 1, 2, 4, 8)
SIZE_P = (0.20, 0.15, 0.20, 0.15, 0.15, 0.15)


def make_trace(n_jobs: int, n_gpus: int, load: float, mean_min: float, seed: int):
    rng = random.Random(seed)
    mean_k = sum(k * p for k, p in zip(SIZES, SIZE_P))
    rate = load * n_gpus / (mean_k * mean_min)  # arrivals per minute for `load` of the cluster's GPU-time
    t, jobs = 0.0, []
    for j in range(n_jobs):
        t += rng.expovariate(rate)
        jobs.append({"id": j, "arrive": t, "k": rng.choices(SIZES, SIZE_P)[0], "base": rng.expovariate(1.0 / mean_min)})
    return jobs


class Node:
    def __init__(self, topo: Topology, slices: int):
        self.topo = topo  # physical view (8 GPUs)
        self.sliced = time_slice(topo, slices)  # what the device plugin advertises on a shared node
        self.s = slices
        self.slot_used: set = set()  # slice ids held (sliced view)

    def gpu_load(self, g: int) -> int:
        return sum(1 for i in range(g * self.s, (g + 1) * self.s) if i in self.slot_used)

    def busy_gpus(self) -> List[int]:
        return [g for g in range(self.topo.n) if self.gpu_load(g) > 0]


class Sim:
    def __init__(self, topos: List[Topology], policy: str, slices: int):
        self.policy = policy
        self.nodes = [Node(t, slices) for t in topos]
        self.pp = PlacementPolicy()
        self.memo: Dict[tuple, Optional[Tuple[Tuple[int, ...], float]]] = {}

    def _whole_on(self, n: int, k: int):
        node = self.nodes[n]
        busy = tuple(node.busy_gpus())
        key = (n, busy, k)
        if key not in self.memo:
            res = None
            if node.topo.n - len(busy) >= k:
                try:
                    pl = select(node.topo, k, used=list(busy), policy=self.pp)
                    res = (tuple(pl.ids), pl.objective + node_packing_term(node.topo.n - len(busy), k, node.topo.n, self.pp))
                except NoFeasiblePlacement:
                    res = None
            self.memo[key] = res
        return self.memo[key]

    def place(self, m: float) -> Optional[Tuple[int, Tuple[int, ...]]]:
        """-> (node, slice ids held) or None."""
        whole = m >= 1 or self.policy == "whole"
        if whole:
            k = max(1, int(math.ceil(m)))
            cands = []
            for n in range(len(self.nodes)):
                r = self._whole_on(n, k)
                if r is not None:
                    cands.append((r[1], n, r[0]))
            if not cands:
                return None
            _, n, gpus = min(cands)
            s = self.nodes[n].s
            return n, tuple(i for g in gpus for i in range(g * s, (g + 1) * s))
        need = max(1, int(math.ceil(m * self.nodes[0].s - 1e-9)))
        if self.policy in ("shares-firstfit", "shares-spread"):
            order = list(range(len(self.nodes)))
            if self.policy == "shares-spread":  # LeastAllocated: the node with the most free slices first
                order.sort(key=lambda n: (len(self.nodes[n].slot_used), n))
            for n in order:
                node = self.nodes[n]
                for g in range(node.topo.n):
                    free = [i for i in range(g * node.s, (g + 1) * node.s) if i not in node.slot_used]
                    if len(free) >= need:
                        return n, tuple(free[:need])
            return None
        best = None  # Fragment best fit across the cluster: the tightest partly used GPU, then a fresh one
        for n, node in enumerate(self.nodes):
            try:
                ids = place_fraction(node.sliced, need, sorted(node.slot_used))
            except NoFeasiblePlacement:
                continue
            g = ids[0] // node.s
            left = node.s - node.gpu_load(g) - need
            key = (0 if node.gpu_load(g) else 1, left, n)
            if best is None or key < best[0]:
                best = (key, n, ids)
        return None if best is None else (best[1], best[2])


def run(topos: List[Topology], trace, policy: str, slices: int, share_slowdown: float = 1.0) -> Dict[str, object]:
    """``share_slowdown``: run-time factor of a fractional job that starts on a GPU another job already
    shares (HBM and L2 stay shared under the CU masks: 1.13 measured on MI355X next to a Llama job,
    ``bench/share_neighbor.py``)."""
    sim = Sim(topos, policy, slices)
    n_gpus = sum(t.n for t in topos)
    events: List[Tuple[float, int, str, int]] = []
    seq = 0
    for j in trace:
        heapq.heappush(events, (j["arrive"], seq, "arrive", j["id"]))
        seq += 1
    pending: List[int] = []
    where: Dict[int, Tuple[int, Tuple[int, ...]]] = {}
    start: Dict[int, float] = {}
    held = 0.0  # GPU-minutes allocated (a whole GPU for a 0.25 job under `whole`)
    runtime: Dict[int, float] = {}
    now = 0.0
    jobs = {j["id"]: j for j in trace}
    while events:
        now, _, kind, jid = heapq.heappop(events)
        if kind == "arrive":
            pending.append(jid)
        else:
            n, ids = where.pop(jid)
            sim.nodes[n].slot_used -= set(ids)
        still = []
        failed_whole, failed_frac = math.inf, math.inf  # nothing at least this big fits until the next event
        for p in pending:
            m = jobs[p]["k"]
            frac = m < 1 and policy != "whole"
            if (frac and m >= failed_frac) or (not frac and math.ceil(m) >= failed_whole):
                still.append(p)
                continue
            pl = sim.place(m)
            if pl is None:
                if frac:
                    failed_frac = min(failed_frac, m)
                else:
                    failed_whole = min(failed_whole, math.ceil(m))
                still.append(p)
                continue
            n, ids = pl
            node = sim.nodes[n]
            shared = len(ids) < slices and node.gpu_load(ids[0] // slices) > 0
            sim.nodes[n].slot_used |= set(ids)
            where[p] = (n, ids)
            start[p] = now
            rt = jobs[p]["base"] * (share_slowdown if shared else 1.0)
            runtime[p] = rt
            held += len(ids) / slices * rt
            heapq.heappush(events, (now + rt, seq, "finish", p))
            seq += 1
        pending = still
    makespan = now
    waits = [start[j["id"]] - j["arrive"] for j in trace]
    frac = [start[j["id"]] - j["arrive"] for j in trace if j["k"] < 1]
    w8 = [start[j["id"]] - j["arrive"] for j in trace if j["k"] == 8]
    useful = sum(j["k"] * j["base"] for j in trace)
    jct = [w + runtime[j["id"]] for w, j in zip(waits, trace)]
    return {"policy": policy, "goodput": round(useful / (n_gpus * makespan), 4), "allocated": round(held / (n_gpus * makespan), 4),
            "makespan_h": round(makespan / 60, 2), "jct_mean_min": round(statistics.mean(jct), 2),
            "wait_mean_min": round(statistics.mean(waits), 2), "wait_frac_mean_min": round(statistics.mean(frac), 2) if frac else None,
            "wait8_mean_min": round(statistics.mean(w8), 2) if w8 else None}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--jobs", type=int, default=4000)
    ap.add_argument("--loads", default="0.9,1.2",
                    help="offered loads: the trace's work as a fraction of the cluster's GPU-time (> 1 = a standing backlog, "
                         "where goodput is the share of the cluster doing useful work)")
    ap.add_argument("--mean-min", type=float, default=60.0)
    ap.add_argument("--slices", type=int, default=4, help="time slices per GPU on shared nodes")
    ap.add_argument("--share-slowdown", type=float, default=1.13,
                    help="run-time factor of a fractional job that starts next to another on its GPU (measured: 1.13)")
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--policies", default=",".join(POLICIES))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    results = []
    summary: Dict[str, Dict[str, Dict[str, float]]] = {}
    for load in [float(x) for x in a.loads.split(",")]:
        for seed in [int(s) for s in a.seeds.split(",")]:
            topos = [Topology.full_mesh(n=8, numa_split=2, link_gbps=76.5, noise=0.05, seed=seed * 1000 + i, node_name=f"node{i}")
                     for i in range(a.nodes)]
            trace = make_trace(a.jobs, 8 * a.nodes, load, a.mean_min, seed)
            for pol in a.policies.split(","):
                r = run(topos, trace, pol, a.slices, a.share_slowdown)
                r["seed"], r["load"] = seed, load
                print(json.dumps(r), flush=True)
                results.append(r)
        per = {}
        for pol in a.policies.split(","):
            rs = [r for r in results if r["policy"] == pol and r["load"] == load]
            per[pol] = {m: round(statistics.mean(r[m] for r in rs), 4)
                        for m in ("goodput", "allocated", "jct_mean_min", "wait_mean_min", "wait_frac_mean_min", "wait8_mean_min",
                                  "makespan_h")}
        base = per.get("whole")
        if base:
            for s in per.values():
                s["goodput_vs_whole"] = round(s["goodput"] / base["goodput"] - 1.0, 4)
                s["jct_vs_whole"] = round(s["jct_mean_min"] / base["jct_mean_min"] - 1.0, 4)
        summary[f"load={load}"] = per
    print(json.dumps({"summary": summary}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"config": vars(a), "summary": summary, "runs": results}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
