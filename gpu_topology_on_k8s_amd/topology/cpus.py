"""CPU lists (Linux ``cpulist`` format, e.g. ``0-47,96-143``) and the GPU<->CPU affinity terms.

Reference: ``design.md:135-147`` breaks a 1-GPU tie by CPU affinity, and Gaia binds each GPU to its
nearest CPU cores (paper p.3 §III.A "GPU and CPU core are automatically bound",
``gaia_gpu_topology_scheduler.md:44-46``).  On an MI355X node each OAM hangs off one socket.
Discovery (``csrc/topo/topo_reader.cpp``) reads, per device, ``/sys/bus/pci/devices/<bdf>/
local_cpulist`` (``GPUInfo.cpu_affinity``) and the trained PCIe link against its capability
(``GPUInfo.pcie_link_ratio``), and per node the NUMA SLIT distances (``Topology.numa_distance``).

* :func:`access_costs` — the per-device ``access`` term of the placement objective for one pod:
  a degraded host link (PCIe trained below x16 / its generation) and a slow HBM stack (k=1 self-copy
  probe) cost extra, and a pod that names the NUMA node its host threads live on
  (``<prefix>/numa-preference``) pays the SLIT distance to each device's socket.  Devices tied on
  links and packing (the ``design.md:135-147`` case) are then ordered by CPU affinity.
* :func:`device_core_slices` / :func:`recommended_cpuset` — Gaia B6 binding: the local cores of a
  socket are split evenly among the devices attached to it (SMT siblings stay together: every range
  of the cpulist is cut at the same fractions), and a pod is recommended the union of its devices'
  slices (``<prefix>/cpuset`` on the pod, ``GTK_CPUSET`` in the container).
* :func:`apply_cpuset` — the binding itself: the training entry point, ``gtk validate`` and
  ``bench.py`` pin their threads to ``GTK_CPUSET`` (or their own device's slice) intersected with
  the container's allowed CPUs, and size the intra-op thread pools to it.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np

__all__ = ["parse_cpulist", "format_cpulist", "device_core_slices", "recommended_cpuset", "apply_cpuset", "bind_workload",
           "access_costs"]


def _ranges(s: str) -> List[Tuple[int, int]]:
    out = []
    for part in (s or "").replace(" ", "").split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.append((int(a), int(b or a)))
    return out


def parse_cpulist(s: str) -> Set[int]:
    out: Set[int] = set()
    for a, b in _ranges(s):
        out.update(range(a, b + 1))
    return out


def try_parse_cpulist(s: str) -> Optional[Set[int]]:
    """:func:`parse_cpulist`, or None for a malformed list (a hand-edited annotation, not a crash)."""
    try:
        out = parse_cpulist(s)
    except ValueError:
        return None
    return out if all(c >= 0 for c in out) else None


def format_cpulist(cpus: Iterable[int]) -> str:
    xs = sorted(set(int(c) for c in cpus))
    if not xs:
        return ""
    runs: List[str] = []
    start = prev = xs[0]
    for c in xs[1:] + [None]:  # type: ignore[list-item]
        if c is not None and c == prev + 1:
            prev = c
            continue
        runs.append(str(start) if start == prev else f"{start}-{prev}")
        if c is not None:
            start = prev = c
    return ",".join(runs)


def device_core_slices(topo) -> Dict[int, Set[int]]:
    """Disjoint core slice per device: devices sharing a ``local_cpulist`` split each of its ranges
    into equal consecutive chunks in device order (chunk sizes differ by at most one core)."""
    key = tuple(g.cpu_affinity for g in topo.gpus)
    memo = getattr(topo, "_core_slices", None)
    if memo is not None and memo[0] == key:
        return memo[1]
    groups: Dict[str, List[int]] = {}
    for g in topo.gpus:
        if g.cpu_affinity:
            groups.setdefault(g.cpu_affinity, []).append(g.index)
    out: Dict[int, Set[int]] = {g.index: set() for g in topo.gpus}
    for cpulist, devs in groups.items():
        m = len(devs)
        for a, b in _ranges(cpulist):
            n = b - a + 1
            for j, d in enumerate(devs):
                lo, hi = a + (n * j) // m, a + (n * (j + 1)) // m
                out[d].update(range(lo, hi))
    try:
        topo._core_slices = (key, out)
    except AttributeError:  # pragma: no cover - slotted stand-ins
        pass
    return out


def recommended_cpuset(topo, ids: Sequence[int]) -> str:
    """Union of the core slices of ``ids`` ('' when discovery could not read the cpulists)."""
    sl = device_core_slices(topo)
    cpus: Set[int] = set()
    for i in ids:
        cpus |= sl.get(int(i), set())
    return format_cpulist(cpus)


def _tasks() -> List[int]:
    """Thread ids of this process (``/proc/self/task``); just this thread where procfs is absent."""
    try:
        return [int(t) for t in os.listdir("/proc/self/task")]
    except OSError:
        return [0]


def apply_cpuset(spec: Optional[str], source: str = "GTK_CPUSET", threads: bool = True,
                 allowed: Optional[Set[int]] = None, setter=None) -> Dict[str, object]:
    """Gaia B6 in the workload: pin this process to ``spec ∩`` the CPUs it may use, and size the
    intra-op thread pools to the result.

    ``spec`` is a cpulist (the pod's ``GTK_CPUSET`` from Allocate, or the recommended slice of the
    process's own device).  The intersection with ``os.sched_getaffinity(0)`` respects the container's
    cgroup cpuset: a recommendation disjoint from it (the kubelet CPU manager gave the pod other
    cores) is reported and not applied.  Every existing thread of the process is moved (threads made
    later inherit the mask), then OpenMP / torch intra-op threads are set to the core count.
    Returns ``{"applied", "source", "requested", "cpus", "n", "reason"}`` for the JSON report lines.
    ``allowed`` / ``setter`` stand in for the OS calls in tests."""
    want = try_parse_cpulist(spec or "")
    have = set(os.sched_getaffinity(0)) if allowed is None else set(allowed)
    rep: Dict[str, object] = {"applied": False, "source": source, "requested": format_cpulist(want or ()), "cpus": "",
                              "n": 0, "reason": ""}
    if want is None:
        rep["requested"] = str(spec)[:200]
        rep["reason"] = "malformed cpulist: not applied"
        return rep
    if not want:
        rep["reason"] = "no cpuset given"
        return rep
    eff = want & have
    if not eff:
        rep["reason"] = f"disjoint from the CPUs this process may use ({format_cpulist(have)})"
        return rep
    set_aff = setter or os.sched_setaffinity
    moved = 0
    for tid in _tasks() if setter is None else [0]:
        try:
            set_aff(tid, eff)
            moved += 1
        except OSError:  # a thread that exited meanwhile
            continue
    if moved == 0:
        rep["reason"] = "sched_setaffinity failed"
        return rep
    if threads:
        os.environ["OMP_NUM_THREADS"] = str(len(eff))
        import sys

        if "torch" in sys.modules:
            sys.modules["torch"].set_num_threads(len(eff))
    rep.update(applied=True, cpus=format_cpulist(eff), n=len(eff), threads_moved=moved)
    return rep


def bind_workload(mode: str = "auto", own: str = "", env: Optional[Dict[str, str]] = None, **kw) -> Dict[str, object]:
    """The cpuset a workload process pins itself to, applied (:func:`apply_cpuset`).

    ``mode``: ``off``; ``env`` = the pod's ``GTK_CPUSET`` only; ``auto`` = ``GTK_CPUSET`` narrowed to
    ``own`` (the slice of this rank's own device, :func:`recommended_cpuset`) where they overlap — a
    k-GPU pod is given the union of its devices' slices, and each rank takes its device's part — else
    ``GTK_CPUSET``, else ``own`` (a bare-node run has no pod allocation)."""
    env = os.environ if env is None else env
    if mode == "off":
        return {"applied": False, "source": "off", "requested": "", "cpus": "", "n": 0, "reason": "--cpu-bind off"}
    pod = env.get("GTK_CPUSET", "")
    if mode == "env":
        return apply_cpuset(pod, "GTK_CPUSET", **kw)
    pod_set, own_set = try_parse_cpulist(pod), try_parse_cpulist(own)
    if pod_set and own_set and pod_set & own_set:
        return apply_cpuset(format_cpulist(pod_set & own_set), "GTK_CPUSET&device-slice", **kw)
    if pod and pod_set is not None:
        return apply_cpuset(pod, "GTK_CPUSET", **kw)
    return apply_cpuset(own, "device-slice" if not pod else "device-slice (GTK_CPUSET malformed)", **kw)


def access_costs(topo, prefer_numa: Optional[Sequence[int]] = None) -> Optional[np.ndarray]:
    """Per-device access cost (0 = ideal) or None when no signal exists (the term is then 0).

    ``pcie``   1 - trained/capable PCIe (speed x width): 0.5 for a Gen5 link trained at x8;
    ``hbm``    relative HBM self-copy shortfall against the node median (k=1 probe);
    ``numa``   2 x (SLIT distance from the preferred NUMA node(s) - 10) / 10: 0 local, 4.4 remote on
               a 2-socket EPYC (SLIT 32), so with the default weights a stated preference outweighs
               anti-fragmentation packing (``w_frag``); without SLIT data a remote socket costs 2.
    """
    n = topo.n
    cost = np.zeros(n)
    have = False
    for g in topo.gpus:
        r = float(getattr(g, "pcie_link_ratio", -1.0))
        if 0.0 < r <= 1.0:
            have = True
            cost[g.index] += 1.0 - r
    hbm = getattr(topo, "hbm_gbps", None)
    if hbm is not None:
        h = np.asarray(hbm, dtype=np.float64)
        ok = np.isfinite(h) & (h > 0)
        if ok.sum() >= 2:
            have = True
            med = float(np.median(h[ok]))
            cost[ok] += np.maximum(0.0, med / h[ok] - 1.0)
    if prefer_numa:
        have = True
        slit = getattr(topo, "numa_distance", None) or {}
        for g in topo.gpus:
            best = None
            for p in prefer_numa:
                row = slit.get(int(p)) if isinstance(slit, dict) else None
                if row is not None and 0 <= g.numa < len(row):
                    d = 2.0 * (row[g.numa] - 10) / 10.0
                else:
                    d = 0.0 if g.numa == int(p) else 2.0
                best = d if best is None else min(best, d)
            cost[g.index] += max(0.0, best or 0.0)
    return cost if have else None
