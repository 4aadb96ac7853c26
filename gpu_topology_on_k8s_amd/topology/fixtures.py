"""Fixture topologies transcribed from the reference (SURVEY.md §4 "Fixture topologies to ship").

* F1 — ``imgs/gpu_topology_on_machine.png``: ``nvidia-smi topo -m`` of an 8-GPU NVLink host.  NV3
  edges 0-1, 0-5, 1-3, 2-3, 2-7, 4-5, 4-6, 6-7 (an 8-cycle); every other pair PHB; CPU affinity
  0-63 for all GPUs.
* F2 — Gaia paper Fig. 3/4 (``reference/gaia_gpu_topology/gpu_topology_tree.png``): the 8-GPU
  resource-access cost tree.
* F3 — Fig. 5 (``gpu_scheduler_sample_1.png``): F2 with GPU4 and GPU6 used.
* F4 — Fig. 7 experiment tree: SOC -> {PXB{GPU0 c2, GPU1 c2}, PIX{GPU2 c1, GPU3 c1}}.
* F5 — Fig. 8(a): F4 with GPU2 used.
* F6 — Fig. 9: F4 with GPU2 fragmented (0.5 then 0.4 then 0.1 requested).
* F7 — 8x MI355X full xGMI mesh (hops 1), NUMA 0-3 / 4-7, optional measured bandwidth + noise.
* F8 — F7 in CPX compute-partition mode: 8 XCPs per GPU, 64 schedulable devices.

``write_fake_kfd_sysfs`` renders F7/F8-shaped KFD topology trees (the layout
``/sys/class/kfd/kfd/topology/nodes/*/{properties,io_links}`` plus ``/sys/class/drm``) so the
native sysfs reader (``csrc/topo/topo_reader.cpp``) is tested without a GPU.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..placement.gaia import CostTree, tree_from_spec
from .model import Topology

__all__ = [
    "f1_nvlink_host", "F2_SPEC", "f2_tree", "f3_tree", "F4_SPEC", "f4_tree", "f5_tree", "f7_mi355x", "f8_mi355x_cpx",
    "write_fake_kfd_sysfs",
]

_F1_NV3 = [(0, 1), (0, 5), (1, 3), (2, 3), (2, 7), (4, 5), (4, 6), (6, 7)]


def f1_nvlink_host() -> Topology:
    n = 8
    m: List[List[str]] = [["PHB"] * n for _ in range(n)]
    for a, b in _F1_NV3:
        m[a][b] = m[b][a] = "NV3"
    t = Topology.from_ref_matrix(m, numa=[0] * n, node_name="f1-nvlink-host")
    for g in t.gpus:
        g.cpu_affinity = "0-63"
    return t


F2_SPEC: Dict[str, object] = {
    "link": "SOC",
    "children": [
        {"link": "PXB", "children": [{"gpu": 6, "cost": 4}, {"gpu": 7, "cost": 4}]},
        {
            "link": "PHB",
            "children": [
                {"link": "PXB", "children": [{"gpu": 4, "cost": 3}, {"gpu": 5, "cost": 3}]},
                {
                    "link": "PXB",
                    "children": [
                        {"link": "PIX", "children": [{"gpu": 0, "cost": 1}, {"gpu": 1, "cost": 1}]},
                        {"link": "PXB", "children": [{"gpu": 2, "cost": 2}, {"gpu": 3, "cost": 2}]},
                    ],
                },
            ],
        },
    ],
}

F4_SPEC: Dict[str, object] = {
    "link": "SOC",
    "children": [
        {"link": "PXB", "children": [{"gpu": 0, "cost": 2}, {"gpu": 1, "cost": 2}]},
        {"link": "PIX", "children": [{"gpu": 2, "cost": 1}, {"gpu": 3, "cost": 1}]},
    ],
}


def f2_tree() -> CostTree:
    return tree_from_spec(F2_SPEC)


def f3_tree() -> CostTree:
    t = f2_tree()
    t.mark_used([4, 6])
    return t


def f4_tree() -> CostTree:
    return tree_from_spec(F4_SPEC)


def f5_tree() -> CostTree:
    t = f4_tree()
    t.mark_used([2])
    return t


def f7_mi355x(link_gbps: Optional[float] = None, noise: float = 0.0, seed: int = 0, n: int = 8) -> Topology:
    return Topology.full_mesh(n=n, numa_split=2, link_gbps=link_gbps, noise=noise, seed=seed, node_name="f7-mi355x")


def f7_degraded(pairs=((0, 1, 0.6),), link_gbps: float = 150.0) -> Topology:
    """F7 with measured links, some degraded: ``(i, j, fraction)`` runs at that fraction of
    ``link_gbps`` (an xGMI link retrained at a lower width, or a flaky one) — the node on which a
    placement's choice is link-bound, unlike a healthy full mesh."""
    t = f7_mi355x()
    bw = np.where(np.eye(t.n, dtype=bool), np.nan, float(link_gbps))
    for i, j, f in pairs:
        bw[i, j] = bw[j, i] = float(link_gbps) * float(f)
    t.set_measured_bw(bw, {"method": "fixture", "degraded": [list(p) for p in pairs]})
    t.node_name = "f7-degraded"
    return t


def f8_mi355x_cpx(link_gbps: Optional[float] = None, noise: float = 0.0, seed: int = 0) -> Topology:
    return Topology.full_mesh(n=8, numa_split=2, link_gbps=link_gbps, noise=noise, seed=seed, node_name="f8-mi355x-cpx",
                              partitions_per_gpu=8)


# ------------------------------------------------------------------------------------ fake sysfs
_KFD_IOLINK_PCIE = 2
_KFD_IOLINK_XGMI = 11


def _props(path: str, kv: Dict[str, object]) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        for k, v in kv.items():
            f.write(f"{k} {v}\n")


def write_fake_kfd_sysfs(
    root: str,
    n_gpus: int = 8,
    sockets: int = 2,
    partitions_per_gpu: int = 1,
    xgmi: bool = True,
    missing_links: Sequence[tuple] = (),
    compute_partition: Optional[str] = None,
    ras: Optional[Dict[int, Dict[str, object]]] = None,
    degraded_pcie: Sequence[int] = (),
    nics: bool = False,
) -> Dict[str, str]:
    """Write a KFD topology tree + DRM tree for an MI355X node under ``root``.

    Returns ``{"kfd": <topology root>, "drm": <drm root>, "pci": <PCI devices root>, "node": <NUMA root>}``
    (PCI: ``local_cpulist`` and PCIe link files of each package's function 0; NUMA: SLIT rows).  KFD node ids: CPUs first
    (0..sockets-1) then one node per schedulable GPU/XCP, as the amdgpu driver enumerates them.
    ``missing_links`` drops direct xGMI io_links between GPU indices (a degraded node).
    ``ras`` writes amdgpu RAS files for device index ``d``: ``{"umc": (ue, ce), "gfx": (ue, ce),
    "bad_pages": n}`` -> ``ras/<block>_err_count`` and ``ras/gpu_vram_bad_pages``.
    ``nics`` lays the PCI devices out as a ``/sys/devices`` hierarchy (one root complex per socket, one
    PCIe switch per package carrying the GPU and an RDMA NIC ``ionic_<package>``, ``pci/<bdf>`` as
    symlinks into it) and adds an ``ib`` root like ``/sys/class/infiniband``.
    """
    kfd = os.path.join(root, "kfd", "topology")
    drm = os.path.join(root, "drm")
    pci = os.path.join(root, "pci")
    numa_root = os.path.join(root, "node")
    cores = 48
    for c in range(sockets):
        nd = os.path.join(numa_root, f"node{c}")
        os.makedirs(nd, exist_ok=True)
        with open(os.path.join(nd, "distance"), "w") as f:
            f.write(" ".join("10" if c == o else "32" for o in range(sockets)) + "\n")
    nodes = os.path.join(kfd, "nodes")
    per_sock = max(1, n_gpus // sockets)
    total = n_gpus * partitions_per_gpu
    for c in range(sockets):
        _props(os.path.join(nodes, str(c), "properties"), {"cpu_cores_count": 64, "simd_count": 0, "mem_banks_count": 1})
    missing = {(min(a, b), max(a, b)) for a, b in missing_links}
    part = compute_partition or {1: "SPX", 2: "DPX", 4: "QPX", 8: "CPX"}.get(partitions_per_gpu, "CPX")
    for d in range(total):
        phys = d // partitions_per_gpu
        xcp = d % partitions_per_gpu
        nid = sockets + d
        sock = min(phys // per_sock, sockets - 1)
        bus = 0x05 + 0x10 * phys
        location_id = (bus << 8) | xcp  # function number distinguishes XCPs of one package
        base = os.path.join(nodes, str(nid))
        _props(
            os.path.join(base, "properties"),
            {
                "cpu_cores_count": 0,
                "simd_count": 1024 // partitions_per_gpu,
                "simd_per_cu": 4,
                "gfx_target_version": 90500,
                "location_id": location_id,
                "domain": 0,
                "unique_id": 0x1000 + 0x100 * phys + xcp,
                "drm_render_minor": 128 + d,
                "local_mem_size": (288 << 30) // partitions_per_gpu,
            },
        )
        links = [(sock, _KFD_IOLINK_PCIE, 20)]
        for e in range(total):
            if e == d:
                continue
            pe = e // partitions_per_gpu
            if pe == phys:
                links.append((sockets + e, _KFD_IOLINK_XGMI, 10))  # same package
                continue
            if xgmi and (min(phys, pe), max(phys, pe)) not in missing:
                links.append((sockets + e, _KFD_IOLINK_XGMI, 15))
        for li, (to, typ, w) in enumerate(links):
            _props(
                os.path.join(base, "io_links", str(li), "properties"),
                {"type": typ, "node_from": nid, "node_to": to, "weight": w, "min_bandwidth": 0,
                 "max_bandwidth": 76800 if typ == _KFD_IOLINK_XGMI else 64000},
            )
        if xcp == 0:
            pdir = os.path.join(pci, f"0000:{bus:02x}:00.0")
            if nics:
                sw = _pcie_switch(root, sock, phys)
                pdir = os.path.join(sw, f"0000:{bus + 1:02x}:00.0", f"0000:{bus:02x}:00.0")
                os.makedirs(pdir, exist_ok=True)
                os.makedirs(pci, exist_ok=True)
                os.symlink(pdir, os.path.join(pci, f"0000:{bus:02x}:00.0"))
                nbus = bus + 2
                ndir = os.path.join(sw, f"0000:{bus + 1:02x}:01.0", f"0000:{nbus:02x}:00.0")
                os.makedirs(os.path.join(ndir, "net", f"enp{nbus}s0"), exist_ok=True)
                with open(os.path.join(ndir, "numa_node"), "w") as f:
                    f.write(f"{sock}\n")
                os.symlink(ndir, os.path.join(pci, f"0000:{nbus:02x}:00.0"))
                ib = os.path.join(root, "infiniband", f"ionic_{phys}")
                os.makedirs(os.path.join(ib, "ports", "1"), exist_ok=True)
                os.symlink(ndir, os.path.join(ib, "device"))
                for name, val in (("state", "4: ACTIVE"), ("rate", "400 Gb/sec (4X NDR)")):
                    with open(os.path.join(ib, "ports", "1", name), "w") as f:
                        f.write(val + "\n")
            os.makedirs(pdir, exist_ok=True)
            a, tot = sock * cores, sockets * cores
            for name, val in (("vendor", "0x1002"), ("local_cpulist", f"{a}-{a + cores - 1},{a + tot}-{a + tot + cores - 1}"),
                              ("current_link_speed", "32.0 GT/s PCIe"), ("max_link_speed", "32.0 GT/s PCIe"),
                              ("current_link_width", str(8 if phys in degraded_pcie else 16)), ("max_link_width", "16")):
                with open(os.path.join(pdir, name), "w") as f:
                    f.write(val + "\n")
        dev = os.path.join(drm, f"renderD{128 + d}", "device")
        os.makedirs(os.path.join(dev, "drm", f"card{d}"), exist_ok=True)
        with open(os.path.join(dev, "current_compute_partition"), "w") as f:
            f.write(part + "\n")
        with open(os.path.join(dev, "current_memory_partition"), "w") as f:
            f.write("NPS1\n")
        for key, val in ((ras or {}).get(d) or {}).items():
            os.makedirs(os.path.join(dev, "ras"), exist_ok=True)
            if key == "bad_pages":
                with open(os.path.join(dev, "ras", "gpu_vram_bad_pages"), "w") as f:
                    f.writelines(f"0x{0x1000 + i:08x} : 0x00001000 : R\n" for i in range(int(val)))
            else:
                ue, ce = val
                with open(os.path.join(dev, "ras", f"{key}_err_count"), "w") as f:
                    f.write(f"ue: {ue}\nce: {ce}\n")
    return {"kfd": kfd, "drm": drm, "pci": pci, "node": numa_root, "ib": os.path.join(root, "infiniband")}


def _pcie_switch(root: str, sock: int, phys: int) -> str:
    """Upstream port of package ``phys``'s PCIe switch: root complex of socket ``sock`` -> root port
    -> switch upstream port (downstream ports 00.0 = GPU, 01.0 = NIC are its children)."""
    rc = 0x80 * sock
    up_bus = 0x05 + 0x10 * phys - 2
    return os.path.join(root, "devices", f"pci0000:{rc:02x}", f"0000:{rc:02x}:{phys + 1:02x}.1", f"0000:{up_bus:02x}:00.0")


def cost_matrix_stats(t: Topology) -> Dict[str, float]:
    off = t.cost[~np.eye(t.n, dtype=bool)]
    return {"min": float(off.min()), "max": float(off.max()), "mean": float(off.mean())}
