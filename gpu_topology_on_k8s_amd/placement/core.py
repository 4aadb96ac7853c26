"""Exact, topology-aware GPU-subset selection and the 0..10 affinity score.

Reference behaviour:
  * ``design.md:131-190`` — subset selection: req==1 picks one free GPU; req>=2 seeds with the
    closest free pair and grows it Prim-style.  ``design.md:188-190`` documents that a tie on the
    seed pair can lock in a worse set.  This module replaces the greedy with an *exact* search over
    all C(n,k) free subsets (n<=8 on an MI355X node: at most 70 subsets), so the tie flaw cannot
    occur.  The greedy is kept in :mod:`.legacy` for parity tests.
  * ``design.md:192-217`` — score in 0..10.  The reference formula is inverted w.r.t. its own mark
    table; here the score is ``10 / max(1, J)`` of a *cost* objective ``J`` where
    lower is better, so a set of nominal xGMI links with no fragmentation penalty scores 10 and the
    score falls monotonically as cost rises.  The literal formula lives in :mod:`.legacy`.
  * Gaia Singular (paper p.5 Alg. 3, ``gaia.md:38-52``): a 1-GPU request prefers a GPU whose
    sibling is already used.  Generalised here as an anti-fragmentation term: allocating into a
    group (NUMA domain; physical GPU when partitioned) that is still *pristine* costs ``w_frag``.

The objective for a candidate set S (|S| = k) is::

    J(S) = comm(S) + w_bottleneck * (bott(S) - comm(S)) + w_span * span(S) + w_frag * frag(S)
           + w_fit * fit(S) + w_access * acc(S)

    comm  = mean pairwise link cost (1.0 = one nominal xGMI link; 1.0 for k == 1)
    bott  = costliest pair in S: a ring all-reduce runs at its slowest link, which the mean dilutes
            (one half-bandwidth link in a 4-set moves the mean by 1/6); equal to comm on uniform sets
    span  = sum over levels of (#groups touched - #groups minimally needed to host k free devices)
    frag  = sum over levels of #pristine groups left partially used
    fit   = sum over levels and touched groups of free_after/size  (best-fit packing)
    acc   = mean per-device access cost (CPU/NUMA affinity hint, design.md:144-145, Gaia B6)
    + w_link_deficit * deficit: how far the set's worst link falls below the best link of its own
      class (link type, hops, on-package or not) on this node, beyond a LINK_DEFICIT_BAND dead band;
      0 on a healthy (banded) node.  A degraded xGMI link slows every collective that crosses it
      (a 2- or 3-GPU ring uses every pair), which NUMA locality (span) or packing do not make up for
      once it is measurably slow
    + w_nic * nicdef, multi-node pods only (``Problem.nic``): NIC domains (device -> its nearest RDMA
      NIC) the set leaves out, min(k, domains with a free device) - domains touched.  A 2-GPU pod of
      a multi-node job on a node with one NIC per socket gets twice the network bandwidth across the
      sockets; on a full xGMI mesh that costs its collectives nothing

The C++ engine (``csrc/placement/engine.cpp``) implements the same objective with branch-and-bound;
``tests/test_placement.py`` checks both agree (hypothesis: native == Python == brute force).
"""
from __future__ import annotations

import itertools
import math
import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..topology.model import Topology

__all__ = ["PlacementPolicy", "Placement", "Problem", "select", "worst", "select_with", "place_fraction", "evaluate",
           "score_from_objective", "node_packing_term", "NoFeasiblePlacement"]

EPS = 1e-9
# a link costlier than the best link of its class by less than this is noise (measurement spread,
# an unbanded matrix): its deficit is 0.  Beyond it the deficit is the excess over the band
LINK_DEFICIT_BAND = 0.10


class NoFeasiblePlacement(RuntimeError):
    pass


@dataclass(frozen=True)
class PlacementPolicy:
    w_span: float = 0.5
    w_frag: float = 0.25
    w_fit: float = 0.05
    w_access: float = 0.1
    w_bottleneck: float = 0.4  # in [0, 1]: blend of mean and worst link (bench/cluster_trace.py)
    w_link_deficit: float = 1.0  # per unit of the worst link's shortfall against its class's best (see LINK_DEFICIT_BAND)
    w_nic: float = 1.0  # per NIC domain a multi-node pod leaves unused (only with Problem.nic)
    tie_break: str = "first"  # "first" (deterministic, lowest ids) | "random"
    exact_limit: int = 200_000  # Python path: max subsets enumerated exactly; above -> greedy + local search
    node_limit: int = 2_000_000  # native path: branch-and-bound node budget; above -> greedy + local search
    # across nodes (the extender's ranking, not the subset search): breaking a pristine node costs
    # w_frag and every device left free on the chosen node w_node_fit / node size — node-level best fit,
    # so small jobs do not scatter over empty nodes that 8-GPU jobs need (bench/cluster_trace.py)
    w_node_fit: float = 0.2
    # CPX/DPX/QPX nodes: treat the XCPs of one physical GPU as a group (pack multi-XCP requests onto
    # one package, keep whole packages pristine) and keep their cheap on-package links.  False =
    # every device is a stand-alone GPU behind xGMI (A/B baseline; SURVEY.md §5.6 --partition-aware)
    partition_aware: bool = True

    def to_dict(self) -> Dict[str, object]:
        return dict(
            w_span=self.w_span, w_frag=self.w_frag, w_fit=self.w_fit, w_access=self.w_access, w_bottleneck=self.w_bottleneck, w_nic=self.w_nic,
            w_link_deficit=self.w_link_deficit,
            w_node_fit=self.w_node_fit,
            tie_break=self.tie_break, exact_limit=self.exact_limit, node_limit=self.node_limit,
            partition_aware=self.partition_aware,
        )

    @classmethod
    def from_dict(cls, d: Dict[str, object]) -> "PlacementPolicy":
        return cls(**{k: v for k, v in d.items() if k in cls.__dataclass_fields__})


@dataclass
class Placement:
    ids: Tuple[int, ...]
    objective: float
    score: float  # 0..10, higher is better
    comm: float
    terms: Dict[str, float] = field(default_factory=dict)
    exact: bool = True

    @property
    def k8s_score(self) -> int:
        """Integer score for ``HostPriority.score`` (0..MaxExtenderPriority=10)."""
        return int(max(0, min(10, round(self.score))))


@dataclass
class Problem:
    """Everything the objective needs, in flat arrays (mirrors the C++ engine's input)."""

    cost: np.ndarray  # n x n
    free: np.ndarray  # bool[n]
    levels: List[np.ndarray]  # group id per device, innermost level first
    access: np.ndarray  # float[n]
    nic: Optional[np.ndarray] = None  # int[n]: NIC domain per device (-1 none); None = not a multi-node pod
    deficit: Optional[np.ndarray] = None  # n x n: link shortfall against its class's best (None = all 0)

    @classmethod
    def from_topology(cls, topo: Topology, used: Sequence[int] = (), access: Optional[Sequence[float]] = None,
                      partition_aware: bool = True, nic_aware: bool = False) -> "Problem":
        n = topo.n
        free = topo.healthy_mask().copy()
        for u in used:
            if 0 <= int(u) < n:
                free[int(u)] = False
        levels = []
        phys = topo.physical
        cost = np.asarray(topo.cost, dtype=np.float64)
        partitioned = len(set(phys.tolist())) < n
        if partitioned and partition_aware:  # XCP -> physical GPU level is meaningful
            levels.append(phys)
        elif partitioned:  # partition-blind: on-package pairs priced like the node's xGMI pairs
            same = (phys[:, None] == phys[None, :]) & ~np.eye(n, dtype=bool)
            cross = ~(phys[:, None] == phys[None, :])
            if cross.any():
                cost = cost.copy()
                cost[same] = float(np.median(cost[cross]))
        levels.append(topo.numa)
        acc = np.zeros(n) if access is None else np.asarray(access, dtype=np.float64)
        return cls(cost=cost, free=free, levels=levels, access=acc, nic=nic_domains(topo) if nic_aware else None,
                   deficit=link_deficit(topo, cost))

    @property
    def n(self) -> int:
        return len(self.free)


def link_deficit(topo: Topology, cost: np.ndarray) -> Optional[np.ndarray]:
    """Per pair: how far its cost exceeds the cheapest link of the same class on this node (link type,
    hops, both ends on one package or not), as a fraction beyond LINK_DEFICIT_BAND; None when no
    link falls short (the common case: a healthy node, or costs from link classes only)."""
    n = topo.n
    if n < 2:
        return None
    same = topo.physical[:, None] == topo.physical[None, :]
    key = (np.asarray(topo.link_type, dtype=np.int64) * 1024 + np.asarray(topo.hops, dtype=np.int64) * 2 + same)
    c = np.asarray(cost, dtype=np.float64)
    ok = np.isfinite(c) & (c > 0) & ~np.eye(n, dtype=bool)
    out = np.zeros((n, n))
    for k in np.unique(key[ok]):
        m = ok & (key == k)
        best = float(c[m].min())
        out[m] = np.maximum(0.0, c[m] / best - 1.0 - LINK_DEFICIT_BAND)
    return out if out.any() else None


def nic_domains(topo: Topology) -> Optional[np.ndarray]:
    """NIC domain per device: the index of its nearest RDMA NIC (``Topology.nearest_nics``), -1 when
    it has none; None when the node published no NICs."""
    if not topo.nics or not topo.gpu_nic:
        return None
    names = [str(x["name"]) for x in topo.nics]
    out = np.full(topo.n, -1, dtype=np.int64)
    for i in range(topo.n):
        near = topo.nearest_nics([i])
        if near:
            out[i] = names.index(near[0])
    return out


def node_packing_term(free_before: int, k: int, size: int, policy: PlacementPolicy = PlacementPolicy()) -> float:
    """Node-level packing cost of putting k devices on a node with ``free_before`` of ``size`` free:
    the same anti-fragmentation (pristine group broken) and best-fit terms as inside a node, one level
    up.  A constant for every subset of one node, so it only ranks nodes against each other."""
    after = free_before - k
    broken = 1.0 if free_before == size and after > 0 else 0.0
    return policy.w_frag * broken + policy.w_node_fit * after / max(1, size)


def score_from_objective(j: float) -> float:
    return 10.0 / max(1.0, j)


def _level_stats(p: Problem):
    """Per level: (group ids array, {g: size}, {g: free_count})."""
    out = []
    for lv in p.levels:
        size: Dict[int, int] = {}
        fre: Dict[int, int] = {}
        for i, g in enumerate(lv.tolist()):
            size[g] = size.get(g, 0) + 1
            fre[g] = fre.get(g, 0) + (1 if p.free[i] else 0)
        out.append((lv, size, fre))
    return out


def _min_groups(free_counts: Sequence[int], k: int) -> int:
    s = 0
    for i, c in enumerate(sorted(free_counts, reverse=True)):
        s += c
        if s >= k:
            return i + 1
    return len(free_counts)


def evaluate(p: Problem, ids: Sequence[int], policy: PlacementPolicy = PlacementPolicy(), _stats=None) -> Tuple[float, Dict[str, float]]:
    ids = list(ids)
    k = len(ids)
    if k >= 2:
        sub = p.cost[np.ix_(ids, ids)]
        comm = float(sub.sum() / (k * (k - 1)))
        bott = float(max(sub[a, b] for a in range(k) for b in range(a + 1, k)))
    else:
        comm = bott = 1.0
    stats = _stats if _stats is not None else _level_stats(p)
    span = frag = fit = 0.0
    for lv, size, fre in stats:
        take: Dict[int, int] = {}
        for i in ids:
            g = int(lv[i])
            take[g] = take.get(g, 0) + 1
        span += len(take) - _min_groups(list(fre.values()), k)
        for g, t in take.items():
            after = fre[g] - t
            if fre[g] == size[g] and after > 0:
                frag += 1
            fit += after / size[g]
    acc = float(np.mean(p.access[ids])) if k else 0.0
    dft = 0.0
    if p.deficit is not None and k >= 2:
        dft = float(p.deficit[np.ix_(ids, ids)].max())
    nicdef = 0.0
    if p.nic is not None and k:
        domains = {int(d) for d, f in zip(p.nic, p.free) if f and d >= 0}
        touched = {int(p.nic[i]) for i in ids if p.nic[i] >= 0}
        nicdef = float(max(0, min(k, len(domains)) - len(touched)))
    j = (comm + policy.w_bottleneck * (bott - comm) + policy.w_span * span + policy.w_frag * frag
         + policy.w_fit * fit + policy.w_access * acc + policy.w_nic * nicdef + policy.w_link_deficit * dft)
    return j, {"comm": comm, "bottleneck": bott, "nic_deficit": nicdef, "span": span, "frag": frag, "fit": fit, "access": acc,
               "link_deficit": dft}


def _greedy_local(p: Problem, k: int, policy: PlacementPolicy, stats) -> Tuple[List[int], float]:
    """Heuristic for very large n (CPX: 64 XCPs): greedy growth from every seed + 1-swap descent."""
    free_ids = [i for i in range(p.n) if p.free[i]]
    best: Optional[List[int]] = None
    best_j = math.inf
    for seed in free_ids:
        cur = [seed]
        while len(cur) < k:
            cand = None
            cj = math.inf
            for c in free_ids:
                if c in cur:
                    continue
                j, _ = evaluate(p, cur + [c], policy, stats)
                if j < cj - EPS:
                    cj, cand = j, c
            cur.append(cand)
        cur_j, _ = evaluate(p, cur, policy, stats)
        improved = True
        while improved:
            improved = False
            outside = [c for c in free_ids if c not in cur]
            for a_pos in range(len(cur)):
                for b in outside:
                    trial = cur.copy()
                    trial[a_pos] = b
                    tj, _ = evaluate(p, trial, policy, stats)
                    if tj < cur_j - EPS:
                        cur, cur_j, improved = trial, tj, True
                        break
                if improved:
                    break
        if cur_j < best_j - EPS or (abs(cur_j - best_j) <= EPS and sorted(cur) < sorted(best)):
            best, best_j = sorted(cur), cur_j
    assert best is not None
    return best, best_j


def _native_engine():
    from .._native import NativeUnavailable, load

    try:
        return load("_placement")
    except NativeUnavailable:
        return None


def _deficit_kw(p: Problem, policy: PlacementPolicy) -> Dict[str, object]:
    """The link-deficit matrix and weight for the native engine (an empty matrix: no link falls short)."""
    d = np.zeros((0, 0)) if p.deficit is None else np.ascontiguousarray(p.deficit, dtype=np.float64)
    return {"deficit": d, "w_link_deficit": policy.w_link_deficit}


def _select_native(mod, p: Problem, k: int, policy: PlacementPolicy, rng: Optional[random.Random] = None) -> Placement:
    args = (np.ascontiguousarray(p.cost, dtype=np.float64), np.ascontiguousarray(p.free, dtype=bool),
            [lv.astype(np.int64).tolist() for lv in p.levels], np.ascontiguousarray(p.access, dtype=np.float64))
    w = (policy.w_span, policy.w_frag, policy.w_fit, policy.w_access)
    ties = policy.tie_break == "random"
    nic = [] if p.nic is None else [int(x) for x in p.nic]
    dk = _deficit_kw(p, policy)
    r = mod.select(*args, int(k), *w, int(policy.node_limit), ties, w_bottleneck=policy.w_bottleneck, nic=nic,
                   w_nic=policy.w_nic, **dk)
    if not r["feasible"]:
        raise NoFeasiblePlacement(f"need {k} free devices")
    if ties and len(r["ties"]) > 1:
        # same draw as the Python enumeration: lexicographic tie list, one rng.choice
        pick = list((rng or random).choice(r["ties"]))
        if pick != list(r["ids"]):
            e = mod.evaluate(*args, pick, *w, w_bottleneck=policy.w_bottleneck, nic=nic, w_nic=policy.w_nic, **dk)
            r = dict(r, ids=pick, objective=e["objective"], terms=e["terms"])
    terms = dict(r["terms"])
    terms["search_nodes"] = float(r["nodes"])
    terms["search_us"] = float(r["micros"])
    return Placement(ids=tuple(int(i) for i in r["ids"]), objective=float(r["objective"]), score=score_from_objective(r["objective"]),
                     comm=terms["comm"], terms=terms, exact=bool(r["exact"]))


def select(
    topo_or_problem,
    k: int,
    used: Sequence[int] = (),
    policy: PlacementPolicy = PlacementPolicy(),
    access: Optional[Sequence[float]] = None,
    rng: Optional[random.Random] = None,
    engine: str = "auto",
    nic_aware: bool = False,
) -> Placement:
    """Choose ``k`` free devices minimising :func:`evaluate`'s objective.

    ``nic_aware``: the pod is part of a multi-node job, so the set should also cover as many RDMA NIC
    domains as it can (the ``w_nic`` term; no effect on nodes without published NICs).
    ``engine``: ``native`` = C++ branch-and-bound (``csrc/placement/engine.cpp``), ``python`` = the
    enumeration below, ``auto`` = native when built.  A random tie-break asks the engine for the
    full lexicographic tie list (ties are pruned only when strictly worse) and draws from it exactly
    as the enumeration does, so both engines return the same set for the same rng state.
    """
    p = (topo_or_problem if isinstance(topo_or_problem, Problem)
         else Problem.from_topology(topo_or_problem, used, access, partition_aware=policy.partition_aware, nic_aware=nic_aware))
    if k <= 0:
        raise ValueError("k must be >= 1")
    free_ids = [i for i in range(p.n) if p.free[i]]
    if len(free_ids) < k:
        raise NoFeasiblePlacement(f"need {k} free devices, have {len(free_ids)}")
    if engine not in ("auto", "native", "python"):
        raise ValueError(engine)
    if engine != "python":
        mod = _native_engine()
        if mod is not None:
            return _select_native(mod, p, k, policy, rng)
        if engine == "native":
            from .._native import load

            load("_placement")  # raises NativeUnavailable with the build command
    stats = _level_stats(p)
    n_subsets = math.comb(len(free_ids), k)
    if n_subsets <= policy.exact_limit:
        best_j = math.inf
        ties: List[Tuple[int, ...]] = []
        for comb in itertools.combinations(free_ids, k):
            j, _ = evaluate(p, comb, policy, stats)
            if j < best_j - EPS:
                best_j, ties = j, [comb]
            elif j <= best_j + EPS:
                ties.append(comb)
        if policy.tie_break == "random" and len(ties) > 1:
            choice = (rng or random).choice(ties)
        else:
            choice = ties[0]
        exact = True
    else:
        lst, best_j = _greedy_local(p, k, policy, stats)
        choice = tuple(lst)
        exact = False
    j, terms = evaluate(p, choice, policy, stats)
    return Placement(ids=tuple(int(c) for c in choice), objective=j, score=score_from_objective(j), comm=terms["comm"], terms=terms, exact=exact)


def _greedy_ascent(p: Problem, k: int, policy: PlacementPolicy, stats) -> List[int]:
    """Python twin of the engine's maximising greedy (growth from every seed + 1-swap ascent)."""
    free_ids = [i for i in range(p.n) if p.free[i]]
    best: Optional[List[int]] = None
    best_j = -math.inf
    for seed in free_ids:
        cur = [seed]
        while len(cur) < k:
            cand, cj = None, -math.inf
            for c in free_ids:
                if c not in cur:
                    j, _ = evaluate(p, cur + [c], policy, stats)
                    if j > cj + EPS:
                        cj, cand = j, c
            cur.append(cand)
        cur_j, _ = evaluate(p, cur, policy, stats)
        improved = True
        while improved:
            improved = False
            for a_pos in range(len(cur)):
                for b in (c for c in free_ids if c not in cur):
                    trial = cur.copy()
                    trial[a_pos] = b
                    tj, _ = evaluate(p, trial, policy, stats)
                    if tj > cur_j + EPS:
                        cur, cur_j, improved = trial, tj, True
                        break
                if improved:
                    break
        cur = sorted(cur)
        if cur_j > best_j + EPS or (abs(cur_j - best_j) <= EPS and cur < best):
            best, best_j = cur, cur_j
    assert best is not None
    return best


def worst(topo: Topology, k: int, used: Sequence[int] = (), policy: PlacementPolicy = PlacementPolicy(),
          engine: str = "auto", access: Optional[Sequence[float]] = None, nic_aware: bool = False) -> Placement:
    """Highest-objective subset (the "worst-topology placement" of BASELINE config 5), scored by
    exactly the objective :func:`select` minimises for the same pod (``access``, and the NIC-coverage
    term when ``nic_aware``: a multi-node job's A/B must not drop the term its placement used).

    Exhaustive while C(free, k) <= ``exact_limit`` in both engines (the native engine then walks every
    subset, so the bound is the same subset budget the Python enumeration uses, not the
    branch-and-bound ``node_limit`` of :func:`select`), otherwise greedy ascent + 1-swap
    (``exact=False``): a CPX node (64 XCPs, k=8) is C(64,8) ~ 4.4e9 subsets, which must never be
    enumerated in a request or a bench start-up."""
    p = Problem.from_topology(topo, used, access, partition_aware=policy.partition_aware, nic_aware=nic_aware)
    free_ids = [i for i in range(p.n) if p.free[i]]
    if len(free_ids) < k:
        raise NoFeasiblePlacement(f"need {k} free devices, have {len(free_ids)}")
    mod = _native_engine() if engine != "python" else None
    if mod is not None:
        args = (np.ascontiguousarray(p.cost, dtype=np.float64), np.ascontiguousarray(p.free, dtype=bool),
                [lv.astype(np.int64).tolist() for lv in p.levels], np.ascontiguousarray(p.access, dtype=np.float64))
        nic = [] if p.nic is None else [int(x) for x in p.nic]
        r = mod.worst(*args, int(k), policy.w_span, policy.w_frag, policy.w_fit, policy.w_access, int(policy.exact_limit),
                      w_bottleneck=policy.w_bottleneck, nic=nic, w_nic=policy.w_nic, **_deficit_kw(p, policy))
        terms = dict(r["terms"])
        terms["search_us"] = float(r["micros"])
        return Placement(ids=tuple(int(i) for i in r["ids"]), objective=float(r["objective"]),
                         score=score_from_objective(r["objective"]), comm=terms["comm"], terms=terms, exact=bool(r["exact"]))
    stats = _level_stats(p)
    if math.comb(len(free_ids), k) <= policy.exact_limit:
        bj, bc = -math.inf, None
        for comb in itertools.combinations(free_ids, k):
            j, _ = evaluate(p, comb, policy, stats)
            if j > bj + EPS:
                bj, bc = j, comb
        exact = True
    else:
        bc, exact = tuple(_greedy_ascent(p, k, policy, stats)), False
    j, terms = evaluate(p, bc, policy, stats)
    return Placement(ids=tuple(bc), objective=j, score=score_from_objective(j), comm=terms["comm"], terms=terms, exact=exact)


def select_with(topo: Topology, k: int, available: Sequence[int], must_include: Sequence[int] = (),
                policy: PlacementPolicy = PlacementPolicy()) -> Tuple[int, ...]:
    """Best ``k`` devices drawn from ``available`` that contain ``must_include`` (kubelet
    ``GetPreferredAllocation`` semantics).  Devices outside ``available`` are treated as used."""
    avail = sorted({int(a) for a in available})
    must = sorted({int(m) for m in must_include})
    if not set(must) <= set(avail):
        raise NoFeasiblePlacement(f"must-include devices {must} are not all available")
    if len(avail) < k or len(must) > k:
        raise NoFeasiblePlacement(f"need {k} of {len(avail)} available devices (must include {must})")
    used = [i for i in range(topo.n) if i not in set(avail)]
    if not must:
        return select(topo, k, used=used, policy=policy).ids
    p = Problem.from_topology(topo, used, partition_aware=policy.partition_aware)
    rest = [a for a in avail if a not in set(must) and p.free[a]]
    r = k - len(must)
    stats = _level_stats(p)
    if math.comb(len(rest), r) <= policy.exact_limit:
        best, bj = None, math.inf
        for comb in itertools.combinations(rest, r):
            cand = tuple(sorted(must + list(comb)))
            j, _ = evaluate(p, cand, policy, stats)
            if j < bj - EPS:
                best, bj = cand, j
        assert best is not None
        return best
    cur = list(must)  # greedy growth around the mandatory devices
    while len(cur) < k:
        c = min((x for x in rest if x not in cur), key=lambda x: evaluate(p, cur + [x], policy, stats)[0])
        cur.append(c)
    return tuple(sorted(cur))


def place_fraction(topo: Topology, k: int, used: Sequence[int] = (), access: Optional[Sequence[float]] = None) -> Tuple[int, ...]:
    """A fraction of ONE physical GPU as ``k`` of its XCP partitions (Gaia Fragment, paper p.4-5 Alg. 2;
    ``gaia_gpu_topology_scheduler.md:32``), the MI355X-native form of a 0<m<1 request: CPX/DPX/QPX
    hardware partitions instead of API interception.

    Candidates are packages already partly in use with >= k free XCPs; the best fit (fewest XCPs
    left over, the author's note on Alg. 2: "closest to m, so the fragment waste is smallest")
    wins.  Without one, the first pristine package is opened.  Ties break on mean access cost, then
    package id.  Raises :class:`NoFeasiblePlacement` when no package can host ``k``."""
    phys = topo.physical
    healthy = topo.healthy_mask()
    usedset = {int(u) for u in used}
    acc = np.zeros(topo.n) if access is None else np.asarray(access, dtype=np.float64)
    pk: Dict[int, List[int]] = {}
    for i in range(topo.n):
        pk.setdefault(int(phys[i]), []).append(i)
    partial, pristine = [], []
    for g, members in sorted(pk.items()):
        free = [i for i in members if healthy[i] and i not in usedset]
        if len(free) < k:
            continue
        take = free[:k]
        key = (len(free) - k, float(np.mean(acc[take])), g)
        (pristine if len(free) == len(members) else partial).append((key, take))
    pool = partial or pristine
    if not pool:
        raise NoFeasiblePlacement(f"no physical GPU has {k} free partitions")
    return tuple(min(pool)[1])
