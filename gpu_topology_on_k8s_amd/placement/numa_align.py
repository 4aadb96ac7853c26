"""Placement on nodes whose kubelet runs the Topology Manager (``--topology-manager-policy`` other than
``none``).

The extender decides a pod's devices (its GROUP) at bind time.  The device plugin then makes the
kubelet allocate them through ``GetPreferredAllocation`` (``design.md:236-246``).  On a node with an
active Topology Manager the kubelet narrows what it offers first.  For every container (scope
``container``, the default) or once per pod (scope ``pod``), the device manager computes NUMA hints:
every set of NUMA nodes whose free devices, plus the devices an init container handed on, cover the
request.  A hint is *preferred* when it is as narrow as the smallest set of NUMA nodes whose devices
(free or not) could hold the request.  The policy merges the hints: the narrowest preferred one wins,
and among equally narrow ones the smallest bitmask (``bitMask.IsNarrowerThan`` compares equal-width
masks as integers, so {1,2} = 0b0110 beats {0,3} = 0b1001: the highest NUMA id decides first).  The policy also decides admission:

* ``best-effort`` always admits;
* ``restricted`` rejects when the winner is not preferred;
* ``single-numa-node`` rejects unless a preferred single-NUMA hint exists.

A rejected pod ends ``Failed`` with reason ``TopologyAffinityError`` and is never retried on that node.
An admitted container's devices then come from the hinted NUMA nodes (``aligned``):

* when the container needs fewer devices than are aligned, the plugin is asked to choose among
  the aligned ones;
* otherwise it gets all of them, and the plugin chooses the rest from all free devices.

An extender that ignores this picks, on a half-used node, GPUs of NUMA node 1 while the kubelet
offers only NUMA node 0's: the GROUP and the container's devices disagree.  Or the extender binds a
pod that a ``single-numa-node`` kubelet rejects for good.  :func:`plan` replays the kubelet's
procedure step by step on the extender's view of the node.  Within each step the placement objective
chooses where the kubelet leaves the choice to the plugin.  It answers the GROUP the kubelet will
allocate, or why the kubelet would reject the pod.

What is not modelled: hints of the CPU and memory managers (a Guaranteed pod with integer CPUs under
the static CPU policy narrows the merged hint further); the ``prefer-closest-numa-nodes`` policy
option (ties between equally narrow hints broken by NUMA distance; ``gtk doctor`` warns when a
kubelet enables it); and which of several reusable devices the
kubelet hands a container (its set iteration order is unspecified; the lowest ids are assumed).  The
device plugin's pod-resources reconcile corrects the annotations when the kubelet chose otherwise.

The device plugin publishes the node's policy and scope as labels (``--topology-manager-policy`` /
``--topology-manager-scope``, or read from the kubelet's config file, ``--kubelet-config``).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass
from typing import Callable, Dict, FrozenSet, List, Mapping, Optional, Sequence, Set, Tuple

from ..topology.model import Topology

__all__ = ["TopologyManager", "TM_POLICIES", "TM_SCOPES", "plan", "best_hint", "read_kubelet_config",
           "tm_from_labels", "tm_labels"]

TM_POLICIES = ("none", "best-effort", "restricted", "single-numa-node")
TM_SCOPES = ("container", "pod")

Hint = Tuple[Optional[FrozenSet[int]], bool]  # (NUMA nodes or None = any, preferred)


@dataclass(frozen=True)
class TopologyManager:
    policy: str = "none"
    scope: str = "container"

    def __post_init__(self):
        if self.policy not in TM_POLICIES:
            raise ValueError(f"topology manager policy must be one of {TM_POLICIES}, got {self.policy!r}")
        if self.scope not in TM_SCOPES:
            raise ValueError(f"topology manager scope must be one of {TM_SCOPES}, got {self.scope!r}")

    @property
    def active(self) -> bool:
        return self.policy != "none"


def tm_labels(tm: TopologyManager, prefix: str) -> Dict[str, str]:
    return {f"{prefix}/topology-manager-policy": tm.policy, f"{prefix}/topology-manager-scope": tm.scope}


def tm_from_labels(labels: Mapping[str, str], prefix: str) -> TopologyManager:
    """The node's Topology Manager as its device plugin published it; ``none`` when absent or unknown."""
    policy = str(labels.get(f"{prefix}/topology-manager-policy", "none"))
    scope = str(labels.get(f"{prefix}/topology-manager-scope", "container"))
    try:
        return TopologyManager(policy, scope)
    except ValueError:
        return TopologyManager()


def read_kubelet_config(path: str) -> TopologyManager:
    """``topologyManagerPolicy`` / ``topologyManagerScope`` of a KubeletConfiguration file (YAML or
    JSON); the kubelet's defaults (``none`` / ``container``) for keys it does not set."""
    import yaml

    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    return TopologyManager(str(cfg.get("topologyManagerPolicy") or "none"), str(cfg.get("topologyManagerScope") or "container"))


def _masks(nodes: Sequence[int]):
    """Every non-empty set of NUMA nodes, narrowest first, lowest ids first within a width (the
    kubelet's ``bitmask.IterateBitMasks`` order)."""
    for width in range(1, len(nodes) + 1):
        for combo in itertools.combinations(sorted(nodes), width):
            yield frozenset(combo)


def _mask_value(mask: FrozenSet[int]) -> int:
    return sum(1 << n for n in mask)


def best_hint(policy: str, request: int, available: Set[int], reusable: Set[int], numa: Mapping[int, int],
              all_devices: Sequence[int]) -> Tuple[Optional[FrozenSet[int]], bool, bool]:
    """(NUMA nodes of the merged hint or None = any, preferred, admitted) for one device request
    (devices with ``numa < 0`` have no topology)."""
    nodes = sorted({n for n in numa.values() if n >= 0})
    if not nodes:
        return None, True, True
    hints: List[Hint] = []
    if len(available | reusable) >= request:
        min_aff = len(nodes)
        found = []
        for mask in _masks(nodes):
            in_mask = sum(1 for d in all_devices if numa.get(d, -1) in mask)
            if in_mask >= request and len(mask) < min_aff:
                min_aff = len(mask)
            if any(numa.get(d, -1) >= 0 and numa[d] not in mask for d in reusable):
                continue
            matching = sum(1 for d in reusable if numa.get(d, -1) >= 0) + sum(1 for d in available if numa.get(d, -1) in mask)
            if matching >= request:
                found.append(mask)
        hints = [(m, len(m) == min_aff) for m in found]
    if policy == "single-numa-node":
        hints = [h for h in hints if h[0] is not None and len(h[0]) == 1 and h[1]]
    everything = frozenset(nodes)
    best: Hint = (everything, False)
    for mask, pref in hints:
        if pref and not best[1]:
            best = (mask, pref)
        elif pref == best[1] and (len(mask), _mask_value(mask)) < (len(best[0]), _mask_value(best[0])):
            best = (mask, pref)
    mask, pref = best
    if policy == "single-numa-node" and mask == everything:
        mask = None
    admit = policy == "best-effort" or pref
    return mask, pref, admit


Choose = Callable[[int, Sequence[int], Sequence[int]], Sequence[int]]


def plan(topo: Topology, used: Sequence[int], steps: Sequence[Tuple[int, str]], tm: TopologyManager,
         choose: Choose, pod_request: Optional[int] = None) -> Tuple[Optional[Tuple[int, ...]], str]:
    """The devices the kubelet will allocate to a pod of ``steps`` (``(count, kind)`` per container in
    admission order, ``kind`` in ``init`` / ``sidecar`` / ``app``) on a node with ``used`` devices
    taken, when the plugin answers every ``GetPreferredAllocation`` with ``choose(k, offered, must)``
    -> (sorted ids, "") or (None, why the kubelet rejects the pod)."""
    numa = {g.index: int(g.numa) for g in topo.gpus}
    all_devices = [g.index for g in topo.gpus]
    free = {g.index for g in topo.gpus if g.healthy} - set(int(u) for u in used)
    pod_alloc: Set[int] = set()
    reuse: Set[int] = set()
    pod_mask: Optional[FrozenSet[int]] = None
    if tm.active and tm.scope == "pod":
        req = pod_request if pod_request is not None else _pod_request(steps)
        pod_mask, pref, ok = best_hint(tm.policy, req, free, set(), numa, all_devices)
        if not ok:
            return None, _why(tm, req, pod_mask, pref)
    for n, kind in steps:
        avail = free - pod_alloc
        mask = pod_mask
        if tm.active and tm.scope == "container":
            mask, pref, ok = best_hint(tm.policy, n, avail, reuse, numa, all_devices)
            if not ok:
                return None, _why(tm, n, mask, pref)
        if len(reuse) >= n:
            got = set(sorted(reuse)[:n])
        else:
            got = set(reuse)
            needed = n - len(got)
            if len(avail) < needed:
                return None, f"requested number of devices unavailable: need {n}, available {len(avail) + len(got)}"
            aligned = {d for d in avail if mask is not None and numa.get(d, -1) in mask} if tm.active else set()
            if needed < len(aligned):
                got = set(choose(n, sorted(aligned | got), sorted(got)))
            else:
                got |= aligned
                if len(got) < n:
                    got = set(choose(n, sorted(avail | got), sorted(got)))
        pod_alloc |= got
        if kind == "init":
            reuse |= got
        else:
            reuse -= got
    return tuple(sorted(pod_alloc)), ""


def _pod_request(steps: Sequence[Tuple[int, str]]) -> int:
    """The pod-level device request (kubelet ``PodLimits``): the larger of the app containers plus
    sidecars, and of each init container with the sidecars started before it."""
    long_lived = 0
    peak = 0
    for n, kind in steps:
        if kind == "init":
            peak = max(peak, long_lived + n)
        elif kind == "sidecar":
            long_lived += n
    app = sum(n for n, kind in steps if kind == "app")
    return max(peak, long_lived + app)


def _why(tm: TopologyManager, n: int, mask, pref: bool) -> str:
    where = "no single NUMA node" if tm.policy == "single-numa-node" else "no preferred NUMA alignment"
    return (f"TopologyAffinityError: the kubelet's topology manager ({tm.policy}, scope {tm.scope}) would reject "
            f"the pod: {where} fits {n} devices")
