"""Why one k-subset beats another: the objective's terms, and the gain they predict.

The placement A/B of the north-star run times the all-reduce on the scheduler's choice and on an
alternative of the same node (``bench.py``, ``bench/train_llama.py``; paper p.7 Figs. 11-12 compare
Gaia with the default kube-scheduler placement).  On a healthy MI355X node every xGMI link lands in one
band (ops/checks.py), so the subsets can differ only by NUMA span and packing, terms that move the
host side (proxies, staging buffers) and later pods, not the links a ring all-reduce runs on.  A
reader of the JSON line must see that before comparing two busBW numbers.  So every compared subset is
reported with:

* the objective ``J`` (placement/core.py ``evaluate``) and the weighted contribution of each term:
  ``comm`` (mean link cost), ``bottleneck`` (worst link over mean), ``link_deficit`` (the worst
  link's shortfall against the best of its class on the node), ``span`` (NUMA / group spread
  beyond the minimum), ``frag`` (pristine groups broken), ``fit`` (packing), ``access`` (host-core
  affinity), ``nic_deficit``;
* its links: the slowest measured link GB/s (or the worst link cost when nothing was measured), the
  link classes and the NUMA nodes it uses;
* against the chosen subset, the terms that separate the two (largest first) and the **predicted
  gain**, a range.  A ring all-reduce moves every byte over every link of its ring, so its busBW
  follows the slowest one.
  - ``predicted_gain``: the ratio of the two subsets' slowest links over all pairs.  This is the
    expectation when RCCL's channels cross every link of the subset. Nothing hands RCCL the measured
    matrix, so it cannot steer round a link that its own detection reports at full width.
  - ``predicted_gain_ring`` (4 to 8 devices): the ratio of the best rings' slowest links
    (``ring_link_gbps``). This is the expectation if RCCL's ring order does avoid the slow link, the
    optimistic model of bench/cluster_trace.py. With 2 or 3 devices every ring uses every pair, so the
    two are equal.
  Both are 1.00 when only host-side terms separate the subsets.

Subsets compared: ``chosen`` (the placement core), ``worst`` (highest objective), and ``default``
(what the kubelet's device manager hands out with no extender and no preferred allocation: it takes
the free devices in set order, modelled here as the lowest free indices).
"""
from __future__ import annotations

import functools
import itertools
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..topology.model import LinkType, Topology
from .core import PlacementPolicy, Problem, evaluate, score_from_objective

__all__ = ["explain_subsets", "default_subset", "TERMS"]

TERMS = ("comm", "bottleneck", "link_deficit", "span", "frag", "fit", "access", "nic_deficit")


def default_subset(topo: Topology, k: int, used: Sequence[int] = ()) -> Optional[List[int]]:
    """The kubelet's choice without the extender: ``k`` free healthy devices in index order."""
    free = [g.index for g in topo.gpus if g.healthy and g.index not in set(used)]
    return sorted(free)[:k] if len(free) >= k else None


def _weighted(terms: Dict[str, float], policy: PlacementPolicy) -> Dict[str, float]:
    return {"comm": terms["comm"], "bottleneck": policy.w_bottleneck * (terms["bottleneck"] - terms["comm"]),
            "link_deficit": policy.w_link_deficit * terms.get("link_deficit", 0.0),
            "span": policy.w_span * terms["span"], "frag": policy.w_frag * terms["frag"], "fit": policy.w_fit * terms["fit"],
            "access": policy.w_access * terms["access"], "nic_deficit": policy.w_nic * terms["nic_deficit"]}


@functools.lru_cache(maxsize=None)
def _rings(k: int) -> np.ndarray:
    """Every ring over positions 0..k-1 once (start fixed at 0, one direction): ((k-1)!/2, k) indices."""
    return np.array([(0,) + p for p in itertools.permutations(range(1, k)) if p[0] < p[-1]], dtype=np.intp)


def _ring_bound(speed: np.ndarray) -> Optional[float]:
    """The slowest link a ring all-reduce over the devices of the k x k ``speed`` matrix must use
    (higher is faster): every pair for 2-3 devices, else the best ring's slowest link (exhaustive up to
    8 devices, every pair beyond that)."""
    k = speed.shape[0]
    if k < 2:
        return None
    if k <= 3 or k > 8:
        return float(speed[~np.eye(k, dtype=bool)].min())
    r = _rings(k)
    return float(speed[r, np.roll(r, -1, axis=1)].min(axis=1).max())


def _links(topo: Topology, ids: Sequence[int]) -> Dict[str, object]:
    ids = list(ids)
    pairs = [(a, b) for i, a in enumerate(ids) for b in ids[i + 1:]]
    bw = topo.bw_gbps
    gbps: Dict[tuple, float] = {}
    if bw is not None:
        for a, b in pairs:
            v = [x for x in (bw[a, b], bw[b, a]) if np.isfinite(x) and x > 0]
            if v:
                gbps[(a, b)] = gbps[(b, a)] = min(v)
    measured = len(gbps) == 2 * len(pairs)
    classes = sorted({LinkType(int(topo.link_type[a, b])).name for a, b in pairs})
    ring = None
    if measured and pairs:
        ring = _ring_bound(np.array([[gbps[(a, b)] if a != b else np.inf for b in ids] for a in ids]))
    ring_cost = _ring_bound(-np.asarray(topo.cost, dtype=float)[np.ix_(ids, ids)]) if pairs else None
    return {"min_link_gbps": round(min(gbps.values()), 2) if measured and pairs else None,
            "ring_link_gbps": round(ring, 2) if ring is not None else None,
            "max_link_cost": round(max((float(topo.cost[a, b]) for a, b in pairs), default=0.0), 6),
            "ring_link_cost": round(-ring_cost, 6) if ring_cost is not None else 0.0,
            "link_classes": classes, "numa_nodes": sorted({int(topo.gpus[i].numa) for i in ids})}


def explain_subsets(topo: Topology, subsets: Dict[str, Optional[Sequence[int]]], policy: PlacementPolicy = PlacementPolicy(),
                    used: Sequence[int] = (), reference: str = "chosen") -> Dict[str, object]:
    """``{name: {...}}`` for every non-empty subset, plus ``vs_<name>`` comparisons against
    ``reference`` (the chosen subset): separating terms and the link-bound predicted gain."""
    p = Problem.from_topology(topo, used)
    out: Dict[str, object] = {}
    for name, ids in subsets.items():
        if not ids:
            continue
        j, terms = evaluate(p, list(ids), policy)
        out[name] = {"ids": [int(i) for i in ids], "objective": round(j, 6), "score": round(score_from_objective(j), 4),
                     "weighted": {t: round(v, 6) for t, v in _weighted(terms, policy).items()}, **_links(topo, ids)}
    ref = out.get(reference)
    if ref is None:
        return out
    for name, e in list(out.items()):
        if name == reference or not isinstance(e, dict):
            continue
        delta = {t: round(e["weighted"][t] - ref["weighted"][t], 6) for t in TERMS}
        sep = [t for t in sorted(TERMS, key=lambda t: -abs(delta[t])) if abs(delta[t]) > 1e-9]
        if ref["min_link_gbps"] and e["min_link_gbps"]:
            gain, basis = ref["min_link_gbps"] / e["min_link_gbps"], "slowest measured link"
            ring_gain = ref["ring_link_gbps"] / e["ring_link_gbps"]
        else:
            gain = e["max_link_cost"] / ref["max_link_cost"] if ref["max_link_cost"] else 1.0
            ring_gain = e["ring_link_cost"] / ref["ring_link_cost"] if ref["ring_link_cost"] else 1.0
            basis = "worst link cost"
        out[f"vs_{name}"] = {"same_devices": sorted(e["ids"]) == sorted(ref["ids"]), "objective_delta": round(e["objective"] - ref["objective"], 6),
                             "separating_terms": {t: delta[t] for t in sep},
                             "predicted_gain": round(gain, 4), "predicted_gain_ring": round(ring_gain, 4), "predicted_basis": basis,
                             "link_terms_separate": any(t in ("comm", "bottleneck", "link_deficit") for t in sep)}
    return out
