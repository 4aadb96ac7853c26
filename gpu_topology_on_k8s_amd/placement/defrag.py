"""Defragmentation planner: which running pods to move so a k-GPU pod fits well somewhere.

Gaia's Singular algorithm (paper p.5 Alg. 3) avoids fragmentation at placement time, and this
framework's objective packs for the same reason, but arrivals and departures still leave free GPUs
scattered: a cluster can hold 8 free GPUs and no node with 8, or no node with a NUMA-local 4-clique.
kube-scheduler's answer is preemption (``extender.preempt``: evict lower-priority pods).  This
module gives an operator the non-destructive alternative: the smallest set of *moves* (pod -> another
node, placed there by the same placement core) after which a node offers ``k`` free devices in a
good placement.  It only plans; executing a move is a restart of the pod elsewhere (delete + the
controller recreates it, or a checkpoint/resume of the job — ``models/checkpoint.py``).

Search, per target node: subsets of its pods in increasing order of moved devices (then count), each
member re-placed on the other nodes largest-first with the exact placement core; the first feasible
subset of each node is its plan, and the plan with the fewest moved devices, then the best objective
for the ``k``-pod, wins.  Nodes whose devices are time slices or XCP partitions are left out (a move
there is a different shape of request).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from ..topology.model import Topology
from .core import NoFeasiblePlacement, PlacementPolicy, select

__all__ = ["Move", "DefragPlan", "plan_defrag"]


@dataclass
class Move:
    pod: str
    src: str
    src_ids: Tuple[int, ...]
    dst: str
    dst_ids: Tuple[int, ...]


@dataclass
class DefragPlan:
    node: str  # where the k-pod then fits
    ids: Tuple[int, ...]  # its placement there
    objective: float
    score: float
    moves: List[Move] = field(default_factory=list)

    @property
    def moved_devices(self) -> int:
        return sum(len(m.src_ids) for m in self.moves)

    def to_dict(self) -> Dict[str, object]:
        return {"node": self.node, "ids": list(self.ids), "objective": round(self.objective, 6), "score": round(self.score, 3),
                "moved_devices": self.moved_devices,
                "moves": [{"pod": m.pod, "from": m.src, "from_ids": list(m.src_ids), "to": m.dst, "to_ids": list(m.dst_ids)}
                          for m in self.moves]}


def _whole_devices(t: Topology) -> bool:
    return all(g.physical == g.index and int(g.shares) <= 1 for g in t.gpus)


def _place(t: Topology, k: int, used: Sequence[int], policy: PlacementPolicy):
    healthy_free = sum(1 for g in t.gpus if g.healthy and g.index not in set(used))
    if healthy_free < k:
        return None
    try:
        return select(t, k, used=sorted(used), policy=policy)
    except NoFeasiblePlacement:
        return None


def plan_defrag(nodes: Dict[str, Topology], pods: Dict[str, Dict[str, Tuple[int, ...]]], k: int,
                policy: Optional[PlacementPolicy] = None, max_moves: int = 3,
                movable: Optional[Sequence[str]] = None, min_score: float = 0.0) -> Optional[DefragPlan]:
    """The cheapest plan that makes a ``k``-device pod placeable, or None.

    ``nodes``: node -> topology; ``pods``: node -> {pod key: device ids it holds} (every pod holding
    devices, so the used sets are exact); ``movable``: pod keys that may be moved (default: all);
    ``min_score``: a placement only counts when its 0..10 score reaches this (e.g. the score of a
    NUMA-local set, so moves are planned for *good* placements, not just any).  A plan with no moves
    means the pod already fits (its best node is returned)."""
    policy = policy or PlacementPolicy()
    movable_set = None if movable is None else set(movable)
    names = [n for n in sorted(nodes) if _whole_devices(nodes[n])]
    used = {n: {i for ids in pods.get(n, {}).values() for i in ids} for n in names}
    best: Optional[DefragPlan] = None

    def better(p: DefragPlan) -> bool:
        if best is None:
            return True
        return (p.moved_devices, len(p.moves), p.objective) < (best.moved_devices, len(best.moves), best.objective)

    def good(pl) -> bool:
        return pl is not None and pl.score >= min_score - 1e-9

    for n in names:  # already placeable: no moves
        pl = _place(nodes[n], k, used[n], policy)
        if good(pl):
            cand = DefragPlan(n, tuple(pl.ids), pl.objective, pl.score)
            if better(cand):
                best = cand
    if best is not None:
        return best
    for n in names:
        t = nodes[n]
        own = [(p, ids) for p, ids in sorted(pods.get(n, {}).items()) if movable_set is None or p in movable_set]
        subsets = [c for r in range(1, min(max_moves, len(own)) + 1) for c in itertools.combinations(own, r)]
        subsets.sort(key=lambda c: (sum(len(ids) for _, ids in c), len(c)))
        for sub in subsets:
            if best is not None and sum(len(ids) for _, ids in sub) > best.moved_devices:
                break
            freed = {i for _, ids in sub for i in ids}
            pl = _place(t, k, used[n] - freed, policy)
            if not good(pl):
                continue
            # re-place the moved pods on the other nodes, largest first, each on its best node
            trial = {m: set(u) for m, u in used.items() if m != n}
            moves: List[Move] = []
            ok = True
            for p, ids in sorted(sub, key=lambda x: -len(x[1])):
                opts = []
                for m in trial:
                    q = _place(nodes[m], len(ids), trial[m], policy)
                    if q is not None:
                        opts.append((q.objective, m, q))
                if not opts:
                    ok = False
                    break
                _, m, q = min(opts, key=lambda o: (o[0], o[1]))
                trial[m] |= set(q.ids)
                moves.append(Move(p, n, tuple(ids), m, tuple(q.ids)))
            if not ok:
                continue
            cand = DefragPlan(n, tuple(pl.ids), pl.objective, pl.score, moves)
            if better(cand):
                best = cand
            break  # this node's cheapest feasible subset found
    return best
