"""Time-sliced GPU shares: Gaia's vGPU (fractional requests) on unpartitioned (SPX) nodes.

Gaia serves a request for 0 < m < 1 of a GPU by its Fragment algorithm (paper p.4-5 Alg. 2,
``reference/gaia_gpu_topology_scheduler.md:32``): the fraction lands on the GPU whose remaining share
fits it most tightly, and the paper's Table II packs 0.5, 0.4 and 0.1 onto one GPU.  On MI355X the
hardware form of that is XCP partitioning (CPX/DPX/QPX, ``placement.core.place_fraction``), but a node
left in SPX mode — the default — has no partitions.  This module gives such a node the same shape in
software: every physical GPU is advertised as ``S`` *time slices* (device ``i*S + j`` is slice ``j``
of GPU ``i``), so

* the kubelet counts shares under their own extended resource (``amd.com/gpu-slice: 4`` on an
  ``S = 10`` node is 0.4 of one GPU; the node offers no ``amd.com/gpu``, which means a whole GPU
  everywhere: Gaia's separate resource pools, docs/SHARES.md) and the pod-annotation contract
  (``ALIYUN_COM_GPU_GROUP`` = slice ids) stays as it is;
* the extender's Fragment path (``<prefix>/gpu-fraction`` + ``place_fraction``) packs fractions onto
  the best-fitting GPU exactly as it packs XCPs of one package;
* Allocate maps slices back to the physical GPU (its render/card nodes once) and tells the container
  its share (``GTK_GPU_FRACTION``).  Slice ``j`` of a GPU owns the ``j``-th ``1/S`` of its compute
  units, and Allocate hands a pod holding part of a GPU ``HSA_CU_MASK`` with its slices' CUs, so the
  ROCm runtime creates every queue of the container on those CUs only: pods sharing a GPU run on
  disjoint CUs (spatial sharing; on MI355X a half mask gives 53 % of the MFMA rate, a quarter 27 %,
  ``profiles/r02_cumask/``; the mask is applied symmetrically over the 8 XCDs, so the pods share the
  L2s).  Like the HBM cap this is cooperative — a container can rewrite its own
  environment — so it keeps well-behaved neighbours apart rather than confining a hostile one.  HBM is shared: the training entry point caps its caching allocator at
  the share (``torch.cuda.set_per_process_memory_fraction``, ``models/train.py``).  CPX/DPX
  partitions remain the form with isolated HBM and L2.

Slices of one GPU are linked ``INTERNAL`` at the GPU's own HBM bandwidth (they share the device);
slices of different GPUs inherit the physical pair's link class, hops, amdsmi weight and measured
bandwidth.
"""
from __future__ import annotations

import copy
import dataclasses
from typing import Dict, List, Sequence

import numpy as np

from .model import GPUInfo, LinkType, Topology

__all__ = ["time_slice", "slices_per_gpu", "physical_group", "share_fractions", "slice_cus", "cu_mask_env"]

#: compute units of an MI355X (8 XCDs x 32) when discovery could not read the count
DEFAULT_CUS = 256


def slices_per_gpu(topo: Topology) -> int:
    """``S`` of a time-sliced node (1 for a node whose devices are whole GPUs or XCPs)."""
    return max((int(g.shares) for g in topo.gpus), default=1)


def time_slice(topo: Topology, slices: int) -> Topology:
    """``topo`` with every GPU advertised as ``slices`` time slices (``slices <= 1``: ``topo`` itself).

    Only whole GPUs can be sliced: a partitioned node (CPX/DPX/QPX) already exposes hardware
    fractions, and slicing its XCPs would need a third hierarchy level the placement core does not
    model, so that raises ``ValueError``."""
    s = int(slices)
    if s <= 1:
        return topo
    if slices_per_gpu(topo) > 1:
        raise ValueError("topology is already time-sliced")
    if any(g.physical != g.index for g in topo.gpus):
        raise ValueError("time slicing needs an unpartitioned (SPX) node; this one exposes XCP partitions")
    n = topo.n
    phys = np.repeat(np.arange(n), s)  # virtual device -> physical GPU
    gpus: List[GPUInfo] = []
    for v, p in enumerate(phys):
        g = topo.gpus[int(p)]
        gpus.append(dataclasses.replace(g, index=v, physical=int(p), shares=s,
                                        uuid=f"{g.uuid}-s{v % s}" if g.uuid else "",
                                        vram_bytes=int(g.vram_bytes) // s))
    same = phys[:, None] == phys[None, :]

    def expand(m):
        return None if m is None else np.asarray(m)[np.ix_(phys, phys)].copy()

    lt = expand(topo.link_type)
    lt[same] = int(LinkType.INTERNAL)
    hops = expand(topo.hops)
    hops[same] = 0
    weight = expand(topo.weight)
    if weight is not None:
        weight[same] = 0.0
    bw = expand(topo.bw_gbps)
    hbm = None if topo.hbm_gbps is None else np.asarray(topo.hbm_gbps, dtype=np.float64)[phys]
    if hbm is not None:  # slices of one GPU exchange data through its own HBM
        bw[same] = np.broadcast_to(hbm[:, None], bw.shape)[same]
    else:
        bw[same] = np.nan
    probe: Dict[str, object] = copy.deepcopy(topo.probe or {})
    mx = probe.get("amdsmi_max_bw_mbps")
    if mx is not None and np.asarray(mx).shape == (n, n):
        probe["amdsmi_max_bw_mbps"] = expand(np.asarray(mx, dtype=np.float64)).tolist()
    for key in ("ingress_all_gbps",):  # per-device lists follow their GPU
        vals = probe.get(key)
        if isinstance(vals, list) and len(vals) == n:
            probe[key] = [vals[int(p)] for p in phys]
    probe["time_slices"] = s
    out = Topology(
        gpus=gpus, link_type=lt, hops=hops, weight=weight, bw_gbps=bw, cost=None,
        ref_gbps=topo.ref_gbps, node_name=topo.node_name, source=topo.source, probe=probe,
        ref_class=expand(topo.ref_class), hbm_gbps=hbm,
        numa_distance=copy.deepcopy(topo.numa_distance), nics=copy.deepcopy(topo.nics),
        gpu_nic=None if topo.gpu_nic is None else [list(topo.gpu_nic[int(p)]) for p in phys],
    )
    derived = copy.deepcopy(topo)
    derived.recompute_cost()
    if not np.allclose(derived.cost, topo.cost):
        # explicitly priced topology (fixtures, reference trees): keep its pair costs between GPUs;
        # slices of one GPU stay at the cheapest cost the recomputation gave them
        cross = ~same
        cost = out.cost.copy()
        cost[cross] = expand(topo.cost)[cross]
        out.cost = np.round(np.maximum(cost, cost.T), 6)
        out.validate()
    return out


def physical_group(topo: Topology, ids: Sequence[int]) -> List[int]:
    """Physical GPUs (ascending, each once) behind the devices ``ids``."""
    return sorted({int(topo.gpus[int(i)].physical) for i in ids})


def share_fractions(topo: Topology, ids: Sequence[int]) -> Dict[int, float]:
    """Physical GPU -> fraction of it that the time slices ``ids`` hold (slices / S)."""
    held: Dict[int, int] = {}
    for i in set(int(x) for x in ids):
        held[int(topo.gpus[i].physical)] = held.get(int(topo.gpus[i].physical), 0) + 1
    s = slices_per_gpu(topo)
    return {p: min(1.0, c / s) for p, c in held.items()}


def slice_cus(topo: Topology, index: int) -> List[int]:
    """Compute units owned by time slice ``index``: the ``j``-th of ``S`` equal runs of its GPU's CU
    indices.  On MI355X the runtime applies a queue CU mask symmetrically over the 8 XCDs (workgroups
    are dealt to every XCD whatever the mask: ``tests/test_gpu_shares.py``), so any ``c`` indices are
    ``c`` CUs spread over all XCDs, and a slice cannot own an XCD's L2; equal runs are as good as any."""
    g = topo.gpus[int(index)]
    s = max(1, int(g.shares))
    c = int(g.cus) if int(g.cus) > 0 else DEFAULT_CUS
    j = sum(1 for h in topo.gpus[:int(index)] if h.physical == g.physical)
    return list(range(j * c // s, (j + 1) * c // s))


def _ranges(xs: Sequence[int]) -> str:
    out, xs = [], sorted(xs)
    i = 0
    while i < len(xs):
        j = i
        while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
            j += 1
        out.append(str(xs[i]) if i == j else f"{xs[i]}-{xs[j]}")
        i = j + 1
    return ",".join(out)


def cu_mask_env(topo: Topology, ids: Sequence[int]) -> str:
    """``HSA_CU_MASK`` for a container holding the time slices ``ids`` ("" when it holds only whole
    GPUs): ``<ordinal>:<cu list>`` per partly held GPU, ``;``-separated, where the ordinal is the GPU's
    position among the container's GPUs (the ROCm runtime enumerates them in PCI order, which is the
    order of the physical indices)."""
    if slices_per_gpu(topo) <= 1:
        return ""
    frac = share_fractions(topo, ids)
    cus = share_cus(topo, ids)
    return ";".join(f"{ordinal}:{_ranges(cus[p])}" for ordinal, p in enumerate(sorted(frac)) if p in cus)


def share_cus(topo: Topology, ids: Sequence[int]) -> Dict[int, List[int]]:
    """Compute units of each partly held physical GPU of the time slices ``ids`` (whole GPUs omitted)."""
    frac = share_fractions(topo, ids)
    return {p: sorted({c for i in ids if topo.gpus[int(i)].physical == p for c in slice_cus(topo, int(i))})
            for p in sorted(frac) if frac[p] < 1.0}


def format_cus(cus: Sequence[int]) -> str:
    """CU list in HSA_CU_MASK syntax ("0-63,128-191")."""
    return _ranges(list(cus))
