"""Topology discovery front-end: amdsmi (native C++), KFD sysfs (native C++) or a fake node.

Reference: ``design.md:57-59`` — "at init the device plugin obtains the GPU information, including
topology, through the nvml package".  Here the native ``_topo`` module provides two real backends
(SURVEY.md §2.A A1); the ``fake`` backend serves tests and the kind-style plumbing config
(BASELINE config 1: "2 fake CPU-backed GPUs via device-plugin stub").
"""
from __future__ import annotations

import logging
import os
from typing import Dict, Optional

import numpy as np

from .._native import NativeUnavailable, load
from .model import DEFAULT_REF_GBPS, GPUInfo, Topology

log = logging.getLogger(__name__)

__all__ = ["discover", "from_native", "fake_topology", "DiscoveryError"]


class DiscoveryError(RuntimeError):
    pass


def from_native(d: Dict[str, object], node_name: str = "", ref_gbps: float = DEFAULT_REF_GBPS) -> Topology:
    gpus = []
    for g in d["gpus"]:
        gpus.append(
            GPUInfo(
                index=int(g["index"]),
                uuid=str(g.get("uuid", "")),
                bdf=str(g.get("bdf", "")),
                numa=max(0, int(g.get("numa", 0))),
                render_minor=int(g.get("render_minor", -1)),
                card=int(g.get("card", -1)),
                kfd_node=int(g.get("kfd_node", -1)),
                physical=int(g.get("physical", -1)),
                partition=str(g.get("partition") or "SPX"),
                memory_partition=str(g.get("memory_partition") or "NPS1"),
                model=str(g.get("model") or "MI355X"),
                gfx=str(g.get("gfx") or "gfx950"),
                vram_bytes=int(g.get("vram_bytes", 0)),
                healthy=bool(g.get("healthy", True)),
                xgmi_links_up=int(g.get("xgmi_links_up", -1)),
                xgmi_links_total=int(g.get("xgmi_links_total", -1)),
                ecc_correctable=int(g.get("ecc_correctable", -1)),
                ecc_uncorrectable=int(g.get("ecc_uncorrectable", -1)),
                ecc_deferred=int(g.get("ecc_deferred", -1)),
                bad_pages=int(g.get("bad_pages", -1)),
                bad_page_threshold=int(g.get("bad_page_threshold", -1)),
                cpu_affinity=str(g.get("cpu_affinity") or ""),
                pcie_link_ratio=float(g.get("pcie_link_ratio", -1.0)),
                cus=int(g.get("cus", -1)),
            )
        )
    lt = np.array(d["link_type"], dtype=np.int32)
    lt = np.maximum(lt, lt.T)  # conservative symmetrisation (worse class wins)
    hops = np.array(d["hops"], dtype=np.int32)
    hops = np.maximum(hops, hops.T)
    weight = np.array(d.get("weight") or np.zeros_like(lt), dtype=np.float64)
    t = Topology(gpus=gpus, link_type=lt, hops=hops, weight=weight, node_name=node_name, source=str(d.get("source", "native")), ref_gbps=ref_gbps)
    nd = d.get("numa_distance") or {}
    if nd:
        t.numa_distance = {int(k): [int(x) for x in v] for k, v in nd.items()}
    if d.get("nics"):
        t.nics = [dict(x) for x in d["nics"]]
        t.gpu_nic = [[int(c) for c in row] for row in d.get("gpu_nic") or []]
    mx = d.get("max_bw_mbps")
    if mx is not None:
        t.probe.setdefault("amdsmi_max_bw_mbps", mx)
    for w in d.get("warnings", []) or []:
        log.warning("topology: %s", w)
    return t


def fake_topology(n: Optional[int] = None, node_name: str = "", **kw) -> Topology:
    n = int(n if n is not None else os.environ.get("GTK_FAKE_GPUS", "8"))
    numa_split = int(kw.pop("numa_split", 2 if n >= 4 else 1))
    return Topology.full_mesh(n=n, numa_split=numa_split, node_name=node_name or "fake-node", **kw)


def discover(
    backend: str = "auto",
    node_name: str = "",
    sysfs_root: str = "/sys/class/kfd/kfd/topology",
    drm_root: str = "/sys/class/drm",
    amdsmi_lib: Optional[str] = None,
    ref_gbps: float = DEFAULT_REF_GBPS,
    fake_n: Optional[int] = None,
    pci_root: str = "/sys/bus/pci/devices",
    node_root: str = "/sys/devices/system/node",
    ib_root: str = "/sys/class/infiniband",
) -> Topology:
    """Discover the node topology.  ``auto`` = amdsmi, then KFD sysfs; never silently fake.
    ``amdsmi_lib`` defaults to ``$GTK_AMDSMI_LIB`` or ``libamd_smi.so`` (the CPU tests point it at the
    stand-in ``bin/libfake_amdsmi.so``)."""
    node_name = node_name or os.environ.get("NODE_NAME", "") or os.uname().nodename
    amdsmi_lib = amdsmi_lib or os.environ.get("GTK_AMDSMI_LIB", "") or "libamd_smi.so"
    if backend == "fake":
        return fake_topology(fake_n, node_name=node_name)
    errors = []
    order = ["amdsmi", "sysfs"] if backend == "auto" else [backend]
    for b in order:
        try:
            topo_mod = load("_topo")
            if b == "amdsmi":
                d = topo_mod.discover_amdsmi(amdsmi_lib, pci_root, node_root, ib_root)
            elif b == "sysfs":
                d = topo_mod.discover_sysfs(sysfs_root, drm_root, pci_root, node_root, ib_root)
            else:
                raise DiscoveryError(f"unknown backend {b!r}")
            if not d["gpus"]:
                raise DiscoveryError(f"{b}: no GPUs found")
            t = from_native(d, node_name=node_name, ref_gbps=ref_gbps)
            log.info("discovered %d devices via %s", t.n, b)
            return t
        except (RuntimeError, NativeUnavailable, DiscoveryError) as e:
            errors.append(f"{b}: {e}")
    raise DiscoveryError("; ".join(errors))
