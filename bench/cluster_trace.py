#!/usr/bin/env python3
"""Cluster-level evaluation: one job trace on a multi-node MI355X cluster under each placement policy.

    python bench/cluster_trace.py [--nodes 16] [--jobs 3000] [--load 0.9] [--out profiles/sched/cluster_trace.json]

Reference: the Gaia paper reports its production effect as "GPU utilization improved by about 10%"
(abstract, p.7 §V; SURVEY.md §6 last rows) without a reproducible setup.  This is a reproducible
stand-in: a discrete-event simulation that drives the real placement code (the same functions the
extender calls) with a synthetic trace, and measures what a cluster operator sees.

* Cluster: ``--nodes`` x 8 MI355X (F7 full mesh, NUMA 0-3 / 4-7).  Node links are measured-style:
  +-5 % noise and ``--degraded`` links per node at half bandwidth (a retrained/flaky xGMI link).
* Jobs: Poisson arrivals sized to ``--load`` of the cluster, 1/2/4/8 GPUs (35/25/20/20 %), base
  run time exponential (mean 60 min).  A multi-GPU job's run time is ``base * (1 + alpha * (f - 1))``
  (``--alpha`` = its communication share) with f the link factor of its placement (``--link-model``:
  ``ring`` = slowest link of the best ring RCCL can build, default; ``bottleneck``; ``mean``) —
  1.0 on nominal xGMI links, 2.0 when a half-bandwidth link cannot be avoided.
* Scheduler: every pending job, in arrival order, is placed as soon as some node fits it (k8s
  schedules pods independently: no gang, no reservation).  Policies:
    exact        this framework: every node's best subset under the placement objective (links,
                 packing, fragmentation); the node with the best objective wins
    gaia         the paper's tree policies (Fragment/Singular/Link), node chosen by objective
    design       the reference design's greedy/Prim subset, node chosen by objective
    k8s-spread   kube-scheduler default (LeastAllocated node) + kubelet's lowest free device ids
    k8s-binpack  MostAllocated node + lowest free ids
* Metrics: mean job completion time (queueing + run; the user-facing number) and its median
  slowdown over the base run time, goodput (the trace's work at nominal link speed / available GPU-time over the makespan:
  the utilisation that did useful work — busy GPU-time alone would credit a policy for slowing
  jobs down on bad links), raw utilisation, makespan, mean / p95 queueing delay, mean run-time
  inflation from links, and the GPU-hours 8-GPU jobs waited while at least 8 GPUs were free
  somewhere (pure fragmentation).
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import random
import statistics
import sys
from typing import Dict, List, Optional, Tuple

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_topology_on_k8s_amd.placement import PlacementPolicy, select  # noqa: E402
from gpu_topology_on_k8s_amd.placement.core import Problem, evaluate, node_packing_term  # noqa: E402
from gpu_topology_on_k8s_amd.placement.gaia import gaia_schedule, tree_from_topology  # noqa: E402
from gpu_topology_on_k8s_amd.placement.legacy import design_farthest_single, design_greedy_select  # noqa: E402
from gpu_topology_on_k8s_amd.topology.model import Topology  # noqa: E402

POLICIES = ("exact", "gaia", "design", "k8s-spread", "k8s-binpack")
SIZES = (1, 2, 4, 8)
SIZE_P = (0.35, 0.25, 0.20, 0.20)


def _tree_node(i: int) -> Topology:
    """The paper's Fig. 3/4 PCIe tree (F2: PIX/PXB/PHB/SOC levels) as a node: link costs 1..4."""
    from gpu_topology_on_k8s_amd.topology import fixtures as fx
    from gpu_topology_on_k8s_amd.topology.model import GPUInfo, LinkType

    tr = fx.f2_tree()
    cost = np.array([[tr.pair_cost(a, b) if a != b else 0.0 for b in range(8)] for a in range(8)], float)
    numa = [0, 0, 0, 0, 0, 0, 1, 1]
    return Topology(gpus=[GPUInfo(index=g, numa=numa[g]) for g in range(8)], link_type=np.full((8, 8), int(LinkType.PCIE)),
                    hops=np.ones((8, 8), int), cost=cost, node_name=f"node{i}")


def make_cluster(n_nodes: int, degraded: int, seed: int, kind: str = "mi355x") -> List[Topology]:
    rng = np.random.default_rng(seed)
    out = []
    if kind != "mi355x":
        from gpu_topology_on_k8s_amd.topology import fixtures as fx

        for i in range(n_nodes):
            t = _tree_node(i) if kind == "pcie-tree" else fx.f1_nvlink_host()
            t.node_name = f"node{i}"
            out.append(t)
        return out
    for i in range(n_nodes):
        t = Topology.full_mesh(n=8, numa_split=2, link_gbps=76.5, noise=0.05, seed=seed * 1000 + i, node_name=f"node{i}")
        bw = np.array(t.bw_gbps, dtype=float)
        pairs = [(a, b) for a in range(8) for b in range(a + 1, 8)]
        for idx in rng.choice(len(pairs), size=degraded, replace=False):
            a, b = pairs[idx]
            bw[a, b] = bw[b, a] = bw[a, b] * 0.5
        t.set_measured_bw(bw, {"method": "synthetic", "degraded_links": degraded})
        out.append(t)
    return out


def make_trace(n_jobs: int, n_gpus: int, load: float, mean_min: float, seed: int):
    rng = random.Random(seed)
    mean_k = sum(k * p for k, p in zip(SIZES, SIZE_P))
    rate = load * n_gpus / (mean_k * mean_min)  # arrivals per minute for `load` offered utilisation
    t, jobs = 0.0, []
    for j in range(n_jobs):
        t += rng.expovariate(rate)
        k = rng.choices(SIZES, SIZE_P)[0]
        jobs.append({"id": j, "arrive": t, "k": k, "base": rng.expovariate(1.0 / mean_min)})
    return jobs


class Sim:
    def __init__(self, topos: List[Topology], policy: str, alpha: float, link_model: str = "ring",
                 pp: Optional[PlacementPolicy] = None, single: str = "objective"):
        self.single = single
        self.topos = topos
        self.policy = policy
        self.alpha = alpha
        self.link_model = link_model
        self._lf: Dict[tuple, float] = {}
        self.pp = pp or PlacementPolicy()
        self.used: List[set] = [set() for _ in topos]
        self.memo: Dict[Tuple[int, Tuple[int, ...], int], Optional[Tuple[Tuple[int, ...], float]]] = {}

    def _choose_on(self, n: int, k: int) -> Optional[Tuple[Tuple[int, ...], float]]:
        """(ids, objective) of ``policy`` on node n for k devices, or None."""
        used = tuple(sorted(self.used[n]))
        key = (n, used, k)
        if key in self.memo:
            return self.memo[key]
        t = self.topos[n]
        res = None
        if 8 - len(used) >= k:
            if self.policy == "exact" and k == 1 and self.single == "farthest":
                # the reference design's rule for one GPU (design.md:135-147): the free device farthest
                # from the others, so the well-linked ones stay together for multi-GPU jobs
                i = design_farthest_single(t.cost, list(used))
                j, _ = evaluate(Problem.from_topology(t, list(used)), [i], self.pp)
                res = ((int(i),), j)
            elif self.policy == "exact":
                pl = select(t, k, used=list(used), policy=self.pp)
                res = (tuple(pl.ids), pl.objective)
            else:
                if self.policy == "gaia":
                    ids = gaia_schedule(tree_from_topology(t, used=list(used)), k)
                elif self.policy == "design":
                    ids = design_greedy_select(t.cost, list(used), k)
                else:  # kubelet default: lowest free device ids
                    ids = [i for i in range(8) if i not in self.used[n]][:k]
                if len(ids) == k:
                    j, _ = evaluate(Problem.from_topology(t, list(used)), ids, self.pp)
                    res = (tuple(sorted(int(i) for i in ids)), j)
        self.memo[key] = res
        return res

    def place(self, k: int) -> Optional[Tuple[int, Tuple[int, ...]]]:
        cands = []
        for n in range(len(self.topos)):
            r = self._choose_on(n, k)
            if r is None:
                continue
            free = 8 - len(self.used[n])
            if self.policy == "k8s-spread":
                key = (-free, n)
            elif self.policy == "k8s-binpack":
                key = (free, n)
            else:  # the extender's node ranking: objective + node-level packing
                key = (r[1] + node_packing_term(free, k, 8, self.pp), n)
            cands.append((key, n, r[0]))
        if not cands:
            return None
        _, n, ids = min(cands)
        return n, ids

    def link_factor(self, n: int, ids: Tuple[int, ...]) -> float:
        """How much slower than on the node's best link the job's collectives run:
        ``ring`` = the best ring's slowest link (assumes RCCL's ring order avoids a bad link whenever
        a Hamiltonian cycle without it exists; nothing tells RCCL the measured matrix, so this is the
        optimistic model: it credits the rival policies' placements as much as possible, so it
        understates this framework's gain), ``bottleneck`` = the set's slowest link (RCCL's channels
        cross every link), ``mean`` = mean pair cost (traffic spread over every link)."""
        if len(ids) < 2:
            return 1.0
        key = (n, ids, self.link_model)
        if key in self._lf:
            return self._lf[key]
        c = self.topos[n].cost
        med = float(np.min(c[~np.eye(8, dtype=bool)]))  # the node's best link = 1.0 (base run time)
        if self.link_model == "mean":
            v = float(np.mean([c[a, b] for a in ids for b in ids if a != b]))
        elif self.link_model == "bottleneck" or len(ids) <= 3:
            v = float(max(c[a, b] for a in ids for b in ids if a != b))
        else:
            import itertools

            first, rest = ids[0], ids[1:]
            v = min(max(c[x, y] for x, y in zip((first,) + perm, perm + (first,)))
                    for perm in itertools.permutations(rest) if perm[0] < perm[-1])
        self._lf[key] = v / med
        return self._lf[key]


def policy_from(weights: str) -> PlacementPolicy:
    """``w_fit=0,w_frag=0.5`` -> the default PlacementPolicy with those weights replaced."""
    import dataclasses

    kw = {}
    for item in filter(None, (x.strip() for x in weights.split(","))):
        name, _, val = item.partition("=")
        if not name.startswith("w_") or not hasattr(PlacementPolicy, name):
            raise SystemExit(f"--weights: unknown weight {name!r}")
        kw[name] = float(val)
    return dataclasses.replace(PlacementPolicy(), **kw)


def run(topos: List[Topology], trace, policy: str, alpha: float, link_model: str = "ring",
        pp: Optional[PlacementPolicy] = None, single: str = "objective") -> Dict[str, object]:
    sim = Sim(topos, policy, alpha, link_model, pp, single)
    n_gpus = 8 * len(topos)
    events: List[Tuple[float, int, str, int]] = []  # (time, seq, kind, job)
    seq = 0
    for j in trace:
        heapq.heappush(events, (j["arrive"], seq, "arrive", j["id"]))
        seq += 1
    pending: List[int] = []
    where: Dict[int, Tuple[int, Tuple[int, ...]]] = {}
    start: Dict[int, float] = {}
    runtime: Dict[int, float] = {}
    busy = 0.0
    frag_wait = 0.0  # GPU-minutes 8-GPU jobs waited while >= 8 GPUs were free cluster-wide
    now = 0.0
    last = 0.0
    jobs = {j["id"]: j for j in trace}
    while events:
        t, _, kind, jid = heapq.heappop(events)
        # fragmentation accounting over [last, t)
        free_total = n_gpus - sum(len(u) for u in sim.used)
        waiting8 = sum(1 for p in pending if jobs[p]["k"] == 8)
        if waiting8 and free_total >= 8:
            frag_wait += waiting8 * 8 * (t - last)
        last = now = t
        if kind == "arrive":
            pending.append(jid)
        else:
            n, ids = where.pop(jid)
            sim.used[n] -= set(ids)
        still = []
        for p in pending:
            pl = sim.place(jobs[p]["k"])
            if pl is None:
                still.append(p)
                continue
            n, ids = pl
            sim.used[n] |= set(ids)
            where[p] = (n, ids)
            start[p] = now
            rt = jobs[p]["base"] * (1.0 + alpha * (sim.link_factor(n, ids) - 1.0))
            runtime[p] = rt
            busy += jobs[p]["k"] * rt
            heapq.heappush(events, (now + rt, seq, "finish", p))
            seq += 1
        pending = still
    makespan = now
    waits = [start[j["id"]] - j["arrive"] for j in trace]
    infl = [runtime[j["id"]] / j["base"] for j in trace if j["k"] > 1 and j["base"] > 0]
    waits8 = [start[j["id"]] - j["arrive"] for j in trace if j["k"] == 8]
    useful = sum(j["k"] * j["base"] for j in trace)  # GPU-minutes of work at nominal link speed
    jct = [start[j["id"]] - j["arrive"] + runtime[j["id"]] for j in trace]
    slow = [(start[j["id"]] - j["arrive"] + runtime[j["id"]]) / j["base"] for j in trace if j["base"] > 1.0]
    return {"policy": policy, "goodput": round(useful / (n_gpus * makespan), 4),
            "utilization": round(busy / (n_gpus * makespan), 4), "makespan_h": round(makespan / 60, 2),
            "jct_mean_min": round(statistics.mean(jct), 2), "jct_slowdown_median": round(statistics.median(slow), 4),
            "wait_mean_min": round(statistics.mean(waits), 2), "wait_p95_min": round(float(np.percentile(waits, 95)), 2),
            "wait8_mean_min": round(statistics.mean(waits8), 2) if waits8 else None,
            "runtime_inflation_mean": round(statistics.mean(infl), 4) if infl else None,
            "frag_wait_gpu_hours": round(frag_wait / 60, 1), "placements_memoized": len(sim.memo)}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nodes", type=int, default=16)
    ap.add_argument("--jobs", type=int, default=3000)
    ap.add_argument("--load", type=float, default=0.9, help="offered load (fraction of the cluster's GPU-time)")
    ap.add_argument("--mean-min", type=float, default=60.0)
    ap.add_argument("--alpha", type=float, default=0.5, help="communication share of a multi-GPU job's step")
    ap.add_argument("--degraded", type=int, default=2, help="half-bandwidth xGMI links per node (mi355x nodes)")
    ap.add_argument("--node-kind", default="mi355x,pcie-tree",
                    help="comma list of: mi355x = 8 x MI355X xGMI full mesh; pcie-tree = the paper's Fig. 3 PCIe tree (its P4 "
                         "testbed's kind of node); nvlink-host = the reference's NV3 ring + PHB host (F1)")
    ap.add_argument("--link-model", default="ring", choices=["ring", "bottleneck", "mean"],
                    help="how a placement's links slow its collectives (Sim.link_factor)")
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--policies", default=",".join(POLICIES))
    ap.add_argument("--weights", default="", help="objective weights for every policy's scoring and node ranking, "
                                                  "e.g. w_fit=0,w_frag=0 (an ablation; default: PlacementPolicy())")
    ap.add_argument("--single", default="objective", choices=["objective", "farthest"],
                    help="exact's choice for 1-GPU jobs: the objective's, or the reference design's farthest device")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    pp = policy_from(a.weights)
    results = []
    summaries = {}
    for kind in a.node_kind.split(","):
        for seed in [int(s) for s in a.seeds.split(",")]:
            topos = make_cluster(a.nodes, a.degraded, seed, kind)
            trace = make_trace(a.jobs, 8 * a.nodes, a.load, a.mean_min, seed)
            for pol in a.policies.split(","):
                r = run(topos, trace, pol, a.alpha, a.link_model, pp, a.single)
                r["seed"], r["node_kind"] = seed, kind
                print(json.dumps(r), flush=True)
                results.append(r)
        summary = {}
        for pol in a.policies.split(","):
            rs = [r for r in results if r["policy"] == pol and r["node_kind"] == kind]
            summary[pol] = {m: round(statistics.mean(r[m] for r in rs), 4)
                            for m in ("goodput", "jct_mean_min", "jct_slowdown_median", "wait_mean_min", "wait_p95_min",
                                      "runtime_inflation_mean", "frag_wait_gpu_hours", "makespan_h")}
        base = summary.get("k8s-spread")
        if base:
            for pol, s in summary.items():
                s["jct_vs_k8s_spread"] = round(s["jct_mean_min"] / base["jct_mean_min"] - 1.0, 4)
                s["goodput_vs_k8s_spread"] = round(s["goodput"] / base["goodput"] - 1.0, 4)
        summaries[kind] = summary
    out = {"config": vars(a), "summary": summaries, "runs": results}
    print(json.dumps({"summary": summaries}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
