"""Gaia resource-access cost tree and its three placement policies.

Reference: Gaia paper (``reference/Gaia Scheduler- ... .pdf``) p.4 "Algorithm framework" + Fig. 4,
Algs. 1-4 (p.4-5); Chinese summary ``reference/gaia_gpu_topology/gaia_gpu_topology_scheduler.md``
lines 11-58; images ``gpu_topology_tree.png`` (Fig. 4), ``gpu_scheduler_sample_1.png`` (Fig. 5),
``gpu_scheduler_algorithm{,_1,_2}``.

Tree semantics (B1):
  * internal node: the link class joining its children (SOC/PHB/PXB/PIX in the paper; on an
    MI355X node: SYS (cross-NUMA) -> XGMI (NUMA domain) -> INTERNAL (XCPs of one package)), a
    ``link_cost`` used when two allocated GPUs meet at this node, and the free-resource count
    (left number in the figures).
  * leaf: one GPU (or one XCP partition) with capacity 1.0, ``used`` in [0, 1] and its access cost
    (right number in the figures).

Policies:
  * :func:`fragment` (Alg. 2, 0 < m < 1): best-fit over partially used leaves with room; else the
    lowest-cost whole GPU.  On MI355X fractions are realised as XCP partitions.
  * :func:`singular` (Alg. 3, m == 1): free leaves whose sibling ("cousin") is fully used, lowest
    access cost; else lowest-cost free leaf (Fig. 5 -> GPU5).
  * :func:`link` (Alg. 4, m > 1): climb from every free leaf to the smallest subtree holding m free
    GPUs (the paper's pseudocode never inserts into S_c — lines 1-8 — this version does), rank
    candidates by the subtree's link cost then the paper's ``m x child access cost``, and allocate
    inside the winner so as to span as few children as possible.

Tie-breaking is either deterministic (lowest index) or random — the paper's Table I reports a
227/273 split between the tied GPU2/GPU3, i.e. random tie-breaking.
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

from ..topology.model import LinkType, Topology

__all__ = ["TreeNode", "CostTree", "gaia_schedule", "fragment", "singular", "link", "tree_from_topology", "tree_from_spec"]

# Paper cost order SOC > PHB > PXB > PIX (gaia.md:16; the paper text's SOC > PXB > PHB > PIX is
# contradicted by its own Fig. 4 — SURVEY §7.4 #7).
REF_LINK_COST = {"SOC": 8.0, "SYS": 8.0, "NODE": 6.0, "PHB": 5.0, "PXB": 4.0, "PIX": 3.0, "PSB": 2.5}


@dataclass(eq=False)
class TreeNode:
    name: str
    link: str = ""  # internal: link class of the subtree root
    link_cost: float = 0.0
    gpu: Optional[int] = None  # leaf only
    access_cost: float = 0.0  # leaf only
    capacity: float = 1.0  # leaf only
    used: float = 0.0  # leaf only
    children: List["TreeNode"] = field(default_factory=list)
    parent: Optional["TreeNode"] = field(default=None, repr=False)

    @property
    def is_leaf(self) -> bool:
        return self.gpu is not None

    @property
    def resources(self) -> float:
        """Left number of the paper's figures: free capacity in this subtree."""
        if self.is_leaf:
            return max(0.0, self.capacity - self.used)
        return sum(c.resources for c in self.children)

    @property
    def free_whole(self) -> int:
        """Number of completely free GPUs in this subtree."""
        if self.is_leaf:
            return 1 if self.used <= 1e-12 else 0
        return sum(c.free_whole for c in self.children)

    def leaves(self) -> List["TreeNode"]:
        if self.is_leaf:
            return [self]
        out: List[TreeNode] = []
        for c in self.children:
            out.extend(c.leaves())
        return out

    def walk(self) -> Iterable["TreeNode"]:
        yield self
        for c in self.children:
            yield from c.walk()

    def siblings(self) -> List["TreeNode"]:
        if self.parent is None:
            return []
        return [c for c in self.parent.children if c is not self]


class CostTree:
    def __init__(self, root: TreeNode):
        self.root = root
        self._link_parents(root, None)
        self.leaf_by_gpu: Dict[int, TreeNode] = {l.gpu: l for l in root.leaves()}

    @staticmethod
    def _link_parents(node: TreeNode, parent: Optional[TreeNode]) -> None:
        node.parent = parent
        for c in node.children:
            CostTree._link_parents(c, node)

    # -------------------------------------------------------------- state
    def mark_used(self, gpus: Iterable[int], amount: float = 1.0) -> None:
        for g in gpus:
            leaf = self.leaf_by_gpu[g]
            if leaf.used + amount > leaf.capacity + 1e-9:
                raise ValueError(f"GPU{g} over-committed")
            leaf.used = min(leaf.capacity, leaf.used + amount)

    def release(self, gpus: Iterable[int], amount: float = 1.0) -> None:
        for g in gpus:
            leaf = self.leaf_by_gpu[g]
            leaf.used = max(0.0, leaf.used - amount)

    def reset(self) -> None:
        for l in self.leaf_by_gpu.values():
            l.used = 0.0

    def used_map(self) -> Dict[int, float]:
        return {g: l.used for g, l in self.leaf_by_gpu.items()}

    def lca(self, a: int, b: int) -> TreeNode:
        pa = []
        n = self.leaf_by_gpu[a]
        while n is not None:
            pa.append(n)
            n = n.parent
        n = self.leaf_by_gpu[b]
        ids = {id(x) for x in pa}
        while n is not None and id(n) not in ids:
            n = n.parent
        assert n is not None
        return n

    def pair_cost(self, a: int, b: int) -> float:
        return 0.0 if a == b else self.lca(a, b).link_cost

    def render(self) -> str:
        lines: List[str] = []

        def rec(n: TreeNode, d: int) -> None:
            if n.is_leaf:
                lines.append("  " * d + f"GPU{n.gpu} [{n.resources:g} | {n.access_cost:g}]")
            else:
                lines.append("  " * d + f"{n.link or n.name} [{n.resources:g} | 0]")
                for c in n.children:
                    rec(c, d + 1)

        rec(self.root, 0)
        return "\n".join(lines)


# ------------------------------------------------------------------ construction helpers
def tree_from_spec(spec) -> CostTree:
    """Nested spec: internal = ``{"link": "PXB", "children": [...]}``; leaf = ``{"gpu": 0, "cost": 2}``.

    Optional keys: ``link_cost`` (defaults from :data:`REF_LINK_COST`), ``used``.
    """

    def build(s, path: str) -> TreeNode:
        if "gpu" in s:
            return TreeNode(name=f"GPU{s['gpu']}", gpu=int(s["gpu"]), access_cost=float(s.get("cost", 0.0)), used=float(s.get("used", 0.0)))
        link = s.get("link", "")
        lc = float(s.get("link_cost", REF_LINK_COST.get(link, 1.0)))
        node = TreeNode(name=s.get("name", path or link), link=link, link_cost=lc)
        node.children = [build(c, f"{path}/{i}") for i, c in enumerate(s["children"])]
        return node

    return CostTree(build(spec, ""))


def tree_from_topology(topo: Topology, used: Sequence[int] = (), numa_penalty: float = 0.1) -> CostTree:
    """MI355X cost tree: root(SYS) -> NUMA domain(XGMI) -> [physical GPU(INTERNAL) ->] device.

    Link costs come from the (measured) cost matrix: the mean pair cost of device pairs whose LCA
    is that node; leaf access cost is the device's mean cost to everything else (so a device with a
    degraded link is less attractive), normalised to [1, 2).
    """
    n = topo.n
    cost = topo.cost
    numa = topo.numa.tolist()
    phys = topo.physical.tolist()
    partitioned = len(set(phys)) < n

    def mean_cost(pairs):
        vals = [cost[i, j] for i, j in pairs]
        return float(sum(vals) / len(vals)) if vals else 0.0

    row = [float(cost[i].sum() / max(1, n - 1)) for i in range(n)]
    lo, hi = (min(row), max(row)) if row else (0.0, 0.0)
    acc = [1.0 + ((r - lo) / (hi - lo) if hi > lo else 0.0) for r in row]

    numa_nodes: List[TreeNode] = []
    for nd in sorted(set(numa)):
        members = [i for i in range(n) if numa[i] == nd]
        if partitioned:
            gpu_nodes = []
            for pg in sorted(set(phys[i] for i in members)):
                xs = [i for i in members if phys[i] == pg]
                pairs = [(a, b) for a in xs for b in xs if a < b]
                leaves = [TreeNode(name=f"GPU{i}", gpu=i, access_cost=acc[i]) for i in xs]
                gpu_nodes.append(TreeNode(name=f"pkg{pg}", link=LinkType.INTERNAL.abbr, link_cost=mean_cost(pairs) or 0.25, children=leaves))
            children = gpu_nodes
        else:
            children = [TreeNode(name=f"GPU{i}", gpu=i, access_cost=acc[i]) for i in members]
        pairs = [(a, b) for a in members for b in members if a < b and phys[a] != phys[b]]
        numa_nodes.append(TreeNode(name=f"numa{nd}", link=LinkType.XGMI.abbr, link_cost=mean_cost(pairs) or 1.0, children=children))
    cross = [(a, b) for a in range(n) for b in range(n) if a < b and numa[a] != numa[b]]
    root_cost = (mean_cost(cross) or 1.0) + numa_penalty
    if len(numa_nodes) == 1:
        root = numa_nodes[0]
    else:
        root = TreeNode(name="node", link=LinkType.PCIE_SYS.abbr if not cross else "SYS", link_cost=root_cost, children=numa_nodes)
    t = CostTree(root)
    t.mark_used([u for u in used if 0 <= u < n])
    return t


# ------------------------------------------------------------------ policies
def _pick(cands: List[TreeNode], key, tie_break: str, rng: Optional[random.Random]) -> TreeNode:
    best = min(key(c) for c in cands)
    ties = [c for c in cands if key(c) == best]
    if tie_break == "random" and len(ties) > 1:
        return (rng or random).choice(ties)
    return ties[0]


def fragment(tree: CostTree, m: float, tie_break: str = "first", rng: Optional[random.Random] = None) -> List[int]:
    """Alg. 2.  Returns the single GPU receiving the fraction ``m`` (0 < m < 1)."""
    if not 0.0 < m < 1.0:
        raise ValueError("fragment requires 0 < m < 1")
    leaves = tree.root.leaves()
    cands = [l for l in leaves if l.used > 1e-12 and m <= l.resources + 1e-12]
    if cands:
        # best fit: the node whose remaining resources are closest to m (author's note on Alg. 2)
        leaf = _pick(cands, lambda l: (round(l.resources, 9), l.access_cost), tie_break, rng)
    else:
        whole = [l for l in leaves if l.used <= 1e-12]
        if not whole:
            return []
        leaf = _pick(whole, lambda l: l.access_cost, tie_break, rng)
    return [leaf.gpu]


def singular(tree: CostTree, tie_break: str = "first", rng: Optional[random.Random] = None) -> List[int]:
    """Alg. 3.  One whole GPU, preferring one whose cousin is already fully used."""
    leaves = [l for l in tree.root.leaves() if l.used <= 1e-12]
    if not leaves:
        return []
    cands = [l for l in leaves if any(s.is_leaf and s.resources <= 1e-12 for s in l.siblings())]
    pool = cands if cands else leaves
    return [_pick(pool, lambda l: l.access_cost, tie_break, rng).gpu]


def _allocate_within(node: TreeNode, m: int, tie_break: str, rng) -> List[int]:
    if node.is_leaf:
        return [node.gpu] if (m == 1 and node.used <= 1e-12) else []
    # a single child that can host everything: recurse into the cheapest / tightest such child
    holders = [c for c in node.children if c.free_whole >= m]
    if holders:
        child = _pick(holders, lambda c: (0.0 if c.is_leaf else c.link_cost, c.free_whole - m, _min_access(c, m)), tie_break, rng)
        return _allocate_within(child, m, tie_break, rng)
    out: List[int] = []
    remaining = m
    order = sorted(node.children, key=lambda c: (-c.free_whole, _min_access(c, c.free_whole)))
    for c in order:
        if remaining == 0:
            break
        take = min(c.free_whole, remaining)
        if take:
            out += _allocate_within(c, take, tie_break, rng)
            remaining -= take
    return out if remaining == 0 else []


def _min_access(node: TreeNode, m: int) -> float:
    costs = sorted(l.access_cost for l in node.leaves() if l.used <= 1e-12)
    return float(sum(costs[:m]))


def link(tree: CostTree, m: int, tie_break: str = "first", rng: Optional[random.Random] = None) -> List[int]:
    """Alg. 4 (corrected).  ``m`` whole GPUs inside the cheapest smallest-enclosing subtree."""
    if m < 2 or int(m) != m:
        raise ValueError("link requires an integer m > 1")
    m = int(m)
    if tree.root.free_whole < m:
        return []
    cands: Dict[int, TreeNode] = {}
    for leaf in tree.root.leaves():
        if leaf.used > 1e-12:
            continue
        n = leaf
        while n is not None and n.free_whole < m:
            n = n.parent
        if n is not None:
            cands[id(n)] = n
    if not cands:
        return []
    # TotalCost_i = m x children.AccessCost (paper line 10), after the subtree's link class
    best = _pick(
        list(cands.values()),
        lambda c: (c.link_cost, m * (_min_access(c, m) / m), c.free_whole - m),
        tie_break,
        rng,
    )
    return sorted(_allocate_within(best, m, tie_break, rng))


def gaia_schedule(tree: CostTree, m: float, tie_break: str = "first", rng: Optional[random.Random] = None, commit: bool = False) -> List[int]:
    """Alg. 1 dispatcher: 0<m<1 -> Fragment, m==1 -> Singular, m>1 -> Link."""
    if m <= 0:
        raise ValueError("m must be > 0")
    if m < 1:
        s = fragment(tree, m, tie_break, rng)
        amount = m
    elif m == 1:
        s = singular(tree, tie_break, rng)
        amount = 1.0
    else:
        if int(m) != m:
            raise ValueError("requests > 1 GPU must be integers (paper p.4: heterogeneous GPUs cannot compute in parallel)")
        s = link(tree, int(m), tie_break, rng)
        amount = 1.0
    if commit and s:
        tree.mark_used(s, amount)
    return s
