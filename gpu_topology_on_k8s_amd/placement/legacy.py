"""The reference design's own selection and score formulas, kept for parity/conformance.

* :func:`design_greedy_select` — ``design.md:149-186``: req==1 returns the first unused device
  (``design.md:154-160``); req>=2 seeds with the unused pair of minimum ``getTopology`` distance
  (``design.md:162-173``) and grows Prim-style by adding the unused device with the minimum summed
  distance to the chosen set (``design.md:180-184``).  The tie flaw described at
  ``design.md:188-190`` is reproduced faithfully (ties resolved "default to the latter").
* :func:`design_farthest_single` — the prose req==1 rule (``design.md:135-147``): the free GPU
  farthest (max summed distance) from all GPUs, ties broken by CPU affinity.
* :func:`legacy_score` — ``design.md:207-216``: ``10 * (1 - sum(marks) / (6 * #pairs))`` with the
  intended denominator.  The design example (marks 1,1,1,2,3,3) gives 6.94.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import numpy as np

from ..topology.model import RefLinkClass, Topology

__all__ = ["legacy_score", "legacy_mark", "design_greedy_select", "design_farthest_single", "legacy_score_of_set"]


def legacy_mark(cls: RefLinkClass, allow_nvlink: bool = False) -> int:
    """Mark table ``design.md:196-203`` (CrossCPU=1 ... SameBoard=6)."""
    if cls >= RefLinkClass.NV1 and not allow_nvlink:
        raise ValueError("the reference assigns no mark to NVLink classes (design.md:41-47 TODO)")
    return int(min(int(cls), 6))


def legacy_score(marks: Sequence[float]) -> float:
    """``10 * (1 - sum(marks) / (6 * len(marks)))`` — 0 pairs scores 10 (single GPU, design.md:17-19)."""
    marks = list(marks)
    if not marks:
        return 10.0
    return 10.0 * (1.0 - float(sum(marks)) / (6.0 * len(marks)))


def legacy_score_literal(marks: Sequence[float]) -> float:
    """The formula exactly as typed at ``design.md:208``: ``10 - 10*sum/6*len`` (left-assoc)."""
    marks = list(marks)
    return 10.0 - 10.0 * float(sum(marks)) / 6.0 * len(marks)


def legacy_score_of_set(topo: Topology, ids: Sequence[int], allow_nvlink: bool = True) -> float:
    if topo.ref_class is None:
        raise ValueError("legacy score needs a reference-taxonomy topology")
    ids = list(ids)
    marks = [legacy_mark(RefLinkClass(int(topo.ref_class[a, b])), allow_nvlink) for i, a in enumerate(ids) for b in ids[i + 1:]]
    return legacy_score(marks)


def design_greedy_select(dist: np.ndarray, used: Sequence[int], req: int) -> List[int]:
    """Reference greedy/Prim selection over a distance matrix (lower = closer)."""
    n = dist.shape[0]
    used_s = set(int(u) for u in used)
    free = [i for i in range(n) if i not in used_s]
    if req <= 0 or len(free) < req:
        return []
    if req == 1:
        return [free[0]]
    best = None
    mn = np.inf
    for a in free:
        for b in free:
            if a == b:
                continue
            d = dist[a, b]
            # "<=" : on a tie the later pair wins ("默认选择后者", design.md:188)
            if d <= mn:
                mn, best = d, [a, b]
    ids = list(best)
    while len(ids) < req:
        cand, cd = None, np.inf
        for c in free:
            if c in ids:
                continue
            s = float(sum(dist[c, x] for x in ids))
            if s < cd:
                cd, cand = s, c
        ids.append(cand)
    return ids


def design_farthest_single(dist: np.ndarray, used: Sequence[int], cpu_affinity: Optional[Callable[[int], float]] = None) -> Optional[int]:
    n = dist.shape[0]
    used_s = set(int(u) for u in used)
    free = [i for i in range(n) if i not in used_s]
    if not free:
        return None
    sums = {i: float(sum(dist[i, j] for j in range(n) if j != i)) for i in free}
    far = max(sums.values())
    ties = [i for i in free if sums[i] == far]
    if len(ties) > 1 and cpu_affinity is not None:
        return min(ties, key=cpu_affinity)
    return ties[0]
