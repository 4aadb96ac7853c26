"""RCCL all-reduce over xGMI on a scheduler-chosen device subset (one process per GPU).

This is the placement validator of SURVEY.md §3.5 in its multi-process form, and the engine of the
repo-root ``bench.py`` (BASELINE.json metric: "RCCL all-reduce bus GB/s on scheduler-chosen k-GPU
subset").  Flow per job:

1. ``torch.distributed`` (backend ``nccl`` = RCCL) provides the rendezvous store, barriers and the
   max-over-ranks timing reduction.
2. Rank 0 discovers the node topology (amdsmi, native) and runs the placement core to pick the
   k-GPU subset; the choice travels to the other ranks through the store.  Every rank binds to
   ``subset[rank]`` — this is what a pod sees after ``Allocate`` mounted its GROUP.
3. The measured collective is a native RCCL communicator (``_rccl.Comm``, ncclCommInitRank with a
   unique id shipped through the same store) issuing out-of-place ``ncclAllReduce`` (nccl-tests
   semantics: algBW = bytes/t, busBW = algBW * 2(k-1)/k).  ``backend="torch"`` uses
   ``dist.all_reduce`` instead, for cross-checking.
"""
from __future__ import annotations

import json
import logging
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

log = logging.getLogger(__name__)

__all__ = ["DistEnv", "choose_subset", "probe_node", "probe_summary", "AllReduceRunner", "bus_factor", "rccl_log_env",
           "rccl_log_summary"]


def bus_factor(k: int) -> float:
    return 2.0 * (k - 1) / k if k > 1 else 0.0


def rccl_log_env(path_prefix: str) -> Dict[str, str]:
    """Environment that makes RCCL write its init/graph log to ``<prefix>.<pid>`` (set before the
    first communicator is created): the transport of every ring edge and the channel counts RCCL
    chose on this node."""
    return {"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,GRAPH", "NCCL_DEBUG_FILE": f"{path_prefix}.%p"}


_RE_COMM = None


def rccl_log_summary(text: str) -> Dict[str, object]:
    """What RCCL decided, from its INFO log: communicators (rank count), channel counts, and how
    every channel edge is carried (``P2P/IPC``, ``P2P/direct pointer``, ``SHM``, ``NET``...)."""
    import re

    global _RE_COMM
    if _RE_COMM is None:
        _RE_COMM = (re.compile(r"nRanks (\d+)"), re.compile(r"(\d+) coll channels"),
                    re.compile(r"Channel \d+/\d+ : \S+ -> \S+ via (.+?)(?: comm 0x\S+)?\s*$"), None)
    r_ranks, r_coll, r_via, _ = _RE_COMM
    comms, channels, via, version = [], [], {}, None
    for line in text.splitlines():
        m = r_ranks.search(line)
        if m and "comm 0x" in line:
            comms.append(int(m.group(1)))
        m = r_coll.search(line)
        if m:
            channels.append(int(m.group(1)))
        m = r_via.search(line)
        if m:
            via[m.group(1)] = via.get(m.group(1), 0) + 1
        if version is None and "version" in line and ("RCCL" in line or "NCCL" in line):
            version = line.split("INFO", 1)[-1].strip()[:80]
    # intra-node rings must ride xGMI peer access (P2P/IPC, P2P/direct pointer); SHM (host staging,
    # e.g. under NCCL_P2P_DISABLE=1) or NET on a single node means the placement's links were bypassed
    non_p2p = {k: v for k, v in via.items() if not k.startswith("P2P")}
    return {"communicators": len(comms), "nranks": sorted(set(comms)), "coll_channels": sorted(set(channels)),
            "edges_via": via, "non_p2p_edges": non_p2p, "p2p_only": bool(via) and not non_p2p, "version": version}


@dataclass
class DistEnv:
    rank: int
    world: int
    local_rank: int
    store: object = None

    @classmethod
    def from_env(cls) -> "DistEnv":
        return cls(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0")))


@dataclass
class SubsetChoice:
    devices: List[int]
    score: float
    objective: float
    source: str
    worst: Optional[List[int]] = None
    worst_score: Optional[float] = None
    placement_ms: float = 0.0
    probed: bool = False
    hip_devices: List[int] = field(default_factory=list)  # HIP ordinal of devices[r] in this process
    worst_hip: Optional[List[int]] = None
    extra: Dict[str, object] = field(default_factory=dict)
    # the kubelet's own choice with no extender (lowest free indices: placement/explain.py), None when
    # it is the chosen set or no distinct k-subset exists
    default: Optional[List[int]] = None
    default_score: Optional[float] = None
    default_hip: Optional[List[int]] = None

    def to_json(self) -> str:
        return json.dumps(self.__dict__)

    @classmethod
    def from_json(cls, s: str) -> "SubsetChoice":
        return cls(**json.loads(s))


def _visible_device_count() -> int:
    import torch

    return int(torch.cuda.device_count())


def probe_node(preset: str = "quick", backend: str = "auto", timeout: float = 150.0):
    """Node-start link probe in a child process (:func:`ops.probe.probe_in_child`)."""
    from ..ops.probe import probe_in_child

    return probe_in_child(preset, backend=backend, timeout=timeout)


def probe_summary(topo, subset: Sequence[int]) -> Dict[str, object]:
    """Compact view of the measured link matrix for the bench JSON line."""
    import numpy as np

    out: Dict[str, object] = {"meta": topo.probe}
    if topo.hbm_gbps is not None:
        out["hbm_copy_gbps"] = [None if not np.isfinite(v) else round(float(v), 1) for v in topo.hbm_gbps]
    bw = topo.bw_gbps
    if bw is None:
        return out
    off = [float(bw[i, j]) for i in range(topo.n) for j in range(topo.n) if i != j and np.isfinite(bw[i, j])]
    if off:
        out["link_read_gbps"] = {"pairs": len(off), "min": round(min(off), 1), "median": round(float(np.median(off)), 1),
                                 "max": round(max(off), 1)}
        out["matrix_gbps"] = [[None if (i == j or not np.isfinite(bw[i, j])) else round(float(bw[i, j]), 1) for j in range(topo.n)]
                              for i in range(topo.n)]
        sub = [float(bw[i, j]) for i in subset for j in subset if i != j and np.isfinite(bw[i, j])]
        if sub:
            out["subset_link_read_gbps"] = {"min": round(min(sub), 1), "max": round(max(sub), 1)}
    ing = (topo.probe or {}).get("ingress_all_gbps")
    if ing:
        out["ingress_all_gbps"] = ing
    from ..ops.probe import ingress_bound

    bound = ingress_bound(topo, subset)
    if bound is not None:
        out["subset_ingress_bound_gbps"] = round(bound, 1)
    return out


def schedule_via_k8s(topo, k: int, node: str = "", timeout: float = 60.0) -> Dict[str, object]:
    """:func:`_schedule_via_k8s` in a daemon thread, bounded by ``timeout`` seconds (raises on expiry):
    the in-process cluster opens sockets and servers, and a stuck one must not stall the job."""
    import threading

    box: Dict[str, object] = {}

    def run():
        try:
            box["ok"] = _schedule_via_k8s(topo, k, node)
        except Exception as e:  # noqa: BLE001 - re-raised in the caller's thread
            box["err"] = e

    th = threading.Thread(target=run, name="gtk-k8s-flow", daemon=True)
    th.start()
    th.join(timeout)
    if th.is_alive():
        raise TimeoutError(f"k8s flow did not finish within {timeout:.0f}s")
    if "err" in box:
        raise box["err"]  # type: ignore[misc]
    return box["ok"]  # type: ignore[return-value]


def _schedule_via_k8s(topo, k: int, node: str = "") -> Dict[str, object]:
    """Place a k-GPU pod through the whole Kubernetes path, in process (``sim.SimCluster``, CPU only):
    the device plugin publishes ``topo`` on a fake apiserver and registers with a fake kubelet over
    gRPC; the mini scheduler calls the extender's ``/filter``, ``/sort`` and ``/bind`` over HTTP;
    the kubelet admits the pod through ``GetPreferredAllocation`` + ``Allocate``.  Returns the
    allocated devices, the pod's GROUP annotation and the flow's latencies."""
    from ..sim import SimCluster

    name = node or topo.node_name or "node0"
    with SimCluster({name: topo}) as c:
        c.submit("allreduce-bench", k)
        r = c.schedule_pending()[0]
        if r.error or not r.allocated:
            raise RuntimeError(f"k8s flow did not place the pod: {r.error or 'no devices allocated'}")
        pa = c.assignment("allreduce-bench")
        return {"devices": [int(i) for i in r.allocated], "node": r.node, "extender_score": r.score,
                "group_annotation": ",".join(str(i) for i in pa.group) if pa else None,
                "assigned": bool(pa.assigned) if pa else None,
                "sched_ms": round(r.sched_ms, 3), "admit_ms": round(r.admit_ms, 3)}


def visible_view(topo, nvis: int, visible_bdfs: Optional[Sequence[str]] = None):
    """(placement topology, DeviceMap, source suffix) for a process that sees ``nvis`` HIP devices.

    The node model keeps its indices (the ``ALIYUN_COM_GPU_GROUP`` numbering) and measured links; the
    devices this process cannot reach (``HIP_VISIBLE_DEVICES``, a pod's device cgroup) are marked
    unavailable in a *copy*, so placement and the in-process k8s flow only pick reachable devices,
    and the map turns the chosen indices into HIP ordinals by PCI address.  Without any address
    match (fake/fixture topologies) the first ``nvis`` indices are taken as ordinals 0..nvis-1; a
    model smaller than what HIP sees is replaced by a full mesh of the visible devices."""
    import copy

    from ..topology.discovery import fake_topology
    from ..topology.identity import DeviceMap

    if visible_bdfs is not None:
        dmap = DeviceMap.for_topology(topo, visible_bdfs)
        nvis = len(visible_bdfs)
    else:
        dmap = DeviceMap.identity(min(topo.n, nvis))
        dmap.n_topology, dmap.n_visible = topo.n, nvis
    suffix = "" if dmap.by_bdf or topo.n == nvis else "->visible-prefix"
    if not dmap.by_bdf and topo.n < nvis:
        log.warning("topology has %d devices but %d are visible to HIP; using a full-mesh model of the visible set", topo.n, nvis)
        return fake_topology(nvis), DeviceMap.identity(nvis), "->visible-mesh"
    hidden = dmap.hidden_indices()
    if hidden:
        topo = copy.deepcopy(topo)
        for i in hidden:
            topo.gpus[i].healthy = False
    return topo, dmap, suffix


def choose_subset(k: int, probe: Optional[str] = None, backend: str = "auto", visible: Optional[int] = None,
                  topology=None, via_k8s: bool = False, visible_bdfs: Optional[Sequence[str]] = None) -> SubsetChoice:
    """Rank-0 side: discover the node, optionally probe links, run the placement core.

    ``visible`` overrides the HIP device count (CPU/gloo runs model a mesh of that many devices, with
    no PCI addresses); otherwise the visible devices' PCI addresses (``visible_bdfs``, queried from
    HIP when None) map the node's topology indices onto HIP ordinals (:func:`visible_view`).
    ``topology`` is an already discovered (and probed) node, e.g. from :func:`probe_node`.
    ``devices`` of the result are node-local topology indices (what GROUP carries); ``hip_devices``
    are what each rank binds to."""
    from ..placement import PlacementPolicy, select, worst
    from ..topology.discovery import DiscoveryError, discover, fake_topology
    from ..topology.identity import DeviceMap, hip_device_bdfs

    if visible is None and visible_bdfs is None:
        visible_bdfs = hip_device_bdfs()
    nvis = len(visible_bdfs) if visible is None else int(visible)
    t0 = time.perf_counter()
    try:
        node = topology if topology is not None else discover(backend)
        topo, dmap, suffix = visible_view(node, nvis, visible_bdfs if visible is None else None)
        source = node.source + suffix
    except DiscoveryError as e:
        log.warning("topology discovery failed (%s); using a full-mesh model of %d visible devices", e, nvis)
        topo, dmap, source = fake_topology(nvis), DeviceMap.identity(nvis), "fallback-mesh"
    probed = bool(topo.probe)
    if probe and not probed:
        from ..ops.probe import probe_topology

        probe_topology(topo, preset=probe, dmap=dmap)
        probed = True
    t1 = time.perf_counter()
    pl = select(topo, k, policy=PlacementPolicy())
    ms = (time.perf_counter() - t1) * 1e3
    n_avail = int(topo.healthy_mask().sum())
    w = worst(topo, k) if k < n_avail else None
    devices, score, objective = list(pl.ids), pl.score, pl.objective
    k8s: Optional[Dict[str, object]] = None
    if via_k8s:
        try:
            k8s = schedule_via_k8s(topo, k)
        except Exception as e:  # noqa: BLE001 - the direct placement stands in, and says so
            log.warning("k8s flow failed (%s); using the placement core directly", e)
            k8s = {"error": str(e)}
        else:
            if sorted(k8s["devices"]) != sorted(devices):
                from ..placement.core import Problem, evaluate, score_from_objective

                objective, _ = evaluate(Problem.from_topology(topo, []), k8s["devices"], PlacementPolicy())
                score = score_from_objective(objective)
            devices = list(k8s["devices"])
    from ..placement.explain import default_subset, explain_subsets
    from ..topology.cpus import recommended_cpuset

    kubelet = default_subset(topo, k)
    terms = explain_subsets(topo, {"chosen": devices, "worst": list(w.ids) if w else None, "default": kubelet})
    # the kubelet would have chosen the same devices: explained (same_devices), nothing to time
    dflt = kubelet if kubelet is not None and sorted(kubelet) != sorted(devices) else None
    # Gaia B6: each rank's share of the node's cores = the slice of its own device (bind_workload)
    cpusets = [recommended_cpuset(topo, [d]) for d in devices]
    return SubsetChoice(
        devices=devices,
        score=round(score, 4),
        objective=round(objective, 6),
        source=source,
        worst=list(w.ids) if w else None,
        worst_score=round(w.score, 4) if w else None,
        placement_ms=round(ms, 4),
        probed=probed,
        hip_devices=[dmap.hip(i) for i in devices],
        worst_hip=[dmap.hip(i) for i in w.ids] if w else None,
        default=dflt,
        default_score=terms["default"]["score"] if dflt else None,
        default_hip=[dmap.hip(i) for i in dflt] if dflt else None,
        extra={"discovery_ms": round((t1 - t0) * 1e3, 2), "node_devices": topo.n, "visible_devices": nvis,
               "placement_terms": terms,
               "default_cpusets": [recommended_cpuset(topo, [d]) for d in dflt] if dflt else None,
               "device_map": dmap.to_dict(), "worst_exact": bool(w.exact) if w else None, "cpusets": cpusets,
               "worst_cpusets": [recommended_cpuset(topo, [d]) for d in w.ids] if w else None,
               **({"probe": probe_summary(topo, devices)} if probed else {}),
               **({"k8s": k8s} if k8s is not None else {})},
    )


class AllReduceRunner:
    """One rank's side of the measured all-reduce (native RCCL comm or torch.distributed)."""

    def __init__(self, env: DistEnv, device: int, nbytes: int, dtype: str = "bf16", backend: str = "native", inplace: bool = False,
                 ctas: Optional[Sequence[int]] = None, tag: str = ""):
        """``ctas = (min, max)`` bounds the RCCL communicator's channel (CTA) count through
        ``ncclConfig_t`` (0 = RCCL's own choice); ``tag`` keeps the unique-id store key of several
        communicators built one after another (bench.py's tuning pass) apart."""
        import torch

        self.env, self.device, self.dtype, self.inplace = env, device, dtype, inplace
        self.backend = backend
        self.comm = None
        self.tensor = None
        if backend == "native":
            from .._native import load

            rccl = load("_rccl")
            key = f"gtk/rccl_uid{tag}"
            if env.rank == 0:
                uid = rccl.unique_id()
                env.store.set(key, uid)
            else:
                uid = env.store.get(key)
            mn, mx = (int(ctas[0]), int(ctas[1])) if ctas else (0, 0)
            self.comm = rccl.Comm(bytes(uid), env.world, env.rank, device, mn, mx)
            self.comm.prepare(int(nbytes), dtype)
            self.nbytes = int(self.comm.bytes)
        elif backend in ("torch", "cpu"):
            tdt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[dtype]
            if backend == "cpu" and tdt != torch.float32:
                tdt = torch.float32  # gloo reduces fp32 natively
            esz = torch.empty((), dtype=tdt).element_size()
            dev = "cpu" if backend == "cpu" else f"cuda:{device}"
            self.tensor = torch.ones(max(1, int(nbytes) // esz), dtype=tdt, device=dev)
            self.nbytes = self.tensor.numel() * esz
            # dist.all_reduce is in place; a 1-rank in-place reduce is a no-op, so for k = 1 each step
            # copies a source buffer first (the out-of-place semantics the native path measures)
            self.src = torch.ones_like(self.tensor) if env.world == 1 and not inplace else None
        else:
            raise ValueError(backend)

    def resize(self, nbytes: int) -> None:
        """Re-target the runner to ``nbytes`` per rank (the size sweep after the headline timing)."""
        if self.comm is not None:
            self.comm.prepare(int(nbytes), self.dtype)
            self.nbytes = int(self.comm.bytes)
            return
        import torch

        esz = self.tensor.element_size()
        self.tensor = torch.ones(max(1, int(nbytes) // esz), dtype=self.tensor.dtype, device=self.tensor.device)
        self.nbytes = self.tensor.numel() * esz
        if self.src is not None:
            self.src = torch.ones_like(self.tensor)

    def check(self) -> int:
        """Exact correctness check of one all-reduce; returns wrong elements on this rank."""
        if self.comm is not None:
            return int(self.comm.check(self.inplace))
        import torch
        import torch.distributed as dist

        x = torch.full((4096,), float(self.env.rank + 1), dtype=self.tensor.dtype, device=self.tensor.device)
        dist.all_reduce(x)
        want = self.env.world * (self.env.world + 1) / 2
        return int((x.float() != want).sum().item())

    def step(self) -> None:
        if self.comm is not None:
            self.comm.step(self.inplace)
        else:
            import torch.distributed as dist

            if self.src is not None:
                self.tensor.copy_(self.src)
            dist.all_reduce(self.tensor)

    def synchronize(self) -> None:
        if self.comm is not None:
            self.comm.synchronize()
        if self.backend == "cpu":
            return
        import torch

        torch.cuda.synchronize(self.device)

    def close(self) -> None:
        if self.comm is not None:
            self.comm.destroy()
            self.comm = None
