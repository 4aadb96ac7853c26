"""CPU lists (Linux ``cpulist`` format, e.g. ``0-47,96-143``) and the GPU<->CPU affinity terms.

Reference: ``design.md:135-147`` breaks a 1-GPU tie by CPU affinity, and Gaia binds each GPU to its
nearest CPU cores (paper p.3 §III.A, ``gaia_gpu_topology_scheduler.md:44-46``).  On an MI355X node
each OAM hangs off one socket: ``/sys/bus/pci/devices/<bdf>/local_cpulist`` names the cores that
reach it without crossing the socket interconnect (read by ``csrc/topo/topo_reader.cpp`` into
``GPUInfo.cpu_affinity``).  Two placement inputs come from it:

* :func:`access_costs` — the per-device ``access`` term of the placement objective: how crowded the
  device's local cores already are (cores recommended to pods bound on the node, from their
  ``<prefix>/cpuset`` annotations), plus a slow-HBM penalty from the k=1 self-copy probe.  A 1-GPU
  request whose candidates tie on links and packing therefore goes to the GPU whose socket has the
  most spare cores.
* :func:`recommended_cpuset` — the cpuset written on the pod at bind (Gaia B6 "GPU and CPU core are
  automatically bound"): the union of the chosen devices' local cores, for the kubelet CPU manager
  or the workload's own pinning (``GTK_CPUSET`` in the container).
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Set

import numpy as np

__all__ = ["parse_cpulist", "format_cpulist", "recommended_cpuset", "access_costs"]


def parse_cpulist(s: str) -> Set[int]:
    out: Set[int] = set()
    for part in (s or "").replace(" ", "").split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


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


def recommended_cpuset(topo, ids: Sequence[int]) -> str:
    """Union of the local cores of ``ids`` ('' when discovery could not read them)."""
    cpus: Set[int] = set()
    for i in ids:
        cpus |= parse_cpulist(topo.gpus[int(i)].cpu_affinity)
    return format_cpulist(cpus)


def access_costs(topo, claimed_cpus: Optional[Iterable[int]] = None) -> Optional[np.ndarray]:
    """Per-device access cost in [0, ~2]: ``claimed`` = fraction of the device's local cores already
    recommended to other pods, ``hbm`` = relative HBM self-copy shortfall against the node median
    (a degraded stack).  None when neither signal exists (the objective's access term is then 0)."""
    n = topo.n
    cost = np.zeros(n)
    have = False
    claimed = set(int(c) for c in (claimed_cpus or ()))
    for g in topo.gpus:
        local = parse_cpulist(g.cpu_affinity)
        if local:
            have = True
            cost[g.index] += len(local & claimed) / len(local)
    hbm = getattr(topo, "hbm_gbps", None)
    if hbm is not None:
        h = np.asarray(hbm, dtype=np.float64)
        ok = np.isfinite(h) & (h > 0)
        if ok.sum() >= 2:
            med = float(np.median(h[ok]))
            have = True
            cost[ok] += np.maximum(0.0, med / h[ok] - 1.0)
    return cost if have else None
