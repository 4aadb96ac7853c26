"""Node GPU topology model.

Reference behaviour (what this replaces, not how):
  * ``design.md:57-74`` — ``gpuTopology map[uint]map[uint]gpuTopologyType``: a pairwise link-type
    map filled from NVML at device-plugin init.  Here the pairwise data are dense ``k x k`` matrices
    (link class, hops, amdsmi link weight, measured GB/s, derived cost) because an MI355X node is a
    full xGMI mesh and the interesting signal is *measured bandwidth*, not the link enum.
  * ``design.md:17-19`` — single-GPU convention: no ``map[0][0]`` entry.  The diagonal of every
    matrix is defined as SELF / 0 hops / 0 cost and is never published as a pair.
  * ``design.md:31-47`` — NVML link taxonomy with an unset "bandwidth weight" column and a TODO
    asking for a justification of the weights.  The AMD model answers the TODO by deriving the
    weight from the HIP p2p probe (``ops/probe.py``): ``cost = ref_gbps / measured_gbps``.

The reference taxonomy (SYS/NODE/PHB/PXB/PIX/PSB/NV1-4) is kept as :class:`RefLinkClass` so that the
reference's fixture topologies (``imgs/gpu_topology_on_machine.png``) and its legacy score
(``design.md:196-216``) can be expressed and reproduced exactly.
"""
from __future__ import annotations

import json
import math
from dataclasses import asdict, dataclass, field
from enum import IntEnum
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "LinkType",
    "RefLinkClass",
    "GPUInfo",
    "Topology",
    "DEFAULT_REF_GBPS",
    "default_link_cost",
]

#: Reference bandwidth (GB/s, one direction, one xGMI link) against which measured link
#: bandwidth is normalised into a cost.  cost = DEFAULT_REF_GBPS / measured.  A nominal
#: MI355X xGMI link is ~153 GB/s bidirectional, i.e. ~76 GB/s per direction.
DEFAULT_REF_GBPS = 76.5


class LinkType(IntEnum):
    """AMD-native link classes (``amdsmi_link_type_t`` + partition/NUMA refinement).

    ``amdsmi.h:1028-1033`` defines INTERNAL / PCIE / XGMI / NOT_APPLICABLE / UNKNOWN.  We refine
    PCIE into same-socket and cross-socket (the reference's NODE/PHB vs SYS split) and add SELF.
    """

    SELF = 0
    INTERNAL = 1  # two XCP partitions of the same physical GPU (on-package Infinity Fabric)
    XGMI = 2  # direct or multi-hop xGMI
    PCIE = 3  # PCIe through the host bridge of one socket
    PCIE_SYS = 4  # PCIe across CPU sockets
    UNKNOWN = 5

    @property
    def abbr(self) -> str:
        return _LT_ABBR[self]

    @property
    def desc(self) -> str:
        return _LT_DESC[self]

    @classmethod
    def from_abbr(cls, abbr: str) -> "LinkType":
        for k, v in _LT_ABBR.items():
            if v == abbr:
                return k
        raise KeyError(abbr)


_LT_ABBR = {
    LinkType.SELF: "X",
    LinkType.INTERNAL: "INTERNAL",
    LinkType.XGMI: "XGMI",
    LinkType.PCIE: "PCIE",
    LinkType.PCIE_SYS: "SYS",
    LinkType.UNKNOWN: "UNKNOWN",
}
_LT_DESC = {
    LinkType.SELF: "Self",
    LinkType.INTERNAL: "Same GPU package",
    LinkType.XGMI: "xGMI",
    LinkType.PCIE: "PCIe host bridge",
    LinkType.PCIE_SYS: "Cross CPU socket",
    LinkType.UNKNOWN: "Unknown",
}


class RefLinkClass(IntEnum):
    """Reference link taxonomy (``design.md:33-44``) with the legacy marks (``design.md:196-203``).

    Values equal the legacy *mark* for the six PCIe classes (CrossCPU=1 ... SameBoard=6).  NVLink
    classes have no mark in the reference (``design.md:41-47`` TODO); they are given 7..10 so they
    order above SameBoard, and :func:`legacy_mark` refuses them unless explicitly allowed.
    """

    SYS = 1  # Cross CPU socket
    NODE = 2  # Same CPU socket
    PHB = 3  # Host PCI bridge
    PXB = 4  # Multiple PCI switches
    PIX = 5  # Single PCI switch
    PSB = 6  # Same board
    NV1 = 7
    NV2 = 8
    NV3 = 9
    NV4 = 10

    @property
    def desc(self) -> str:
        return _REF_DESC[self]

    def to_link_type(self) -> LinkType:
        if self >= RefLinkClass.NV1:
            return LinkType.XGMI  # the point-to-point GPU fabric class
        if self == RefLinkClass.SYS:
            return LinkType.PCIE_SYS
        return LinkType.PCIE

    def nominal_cost(self) -> float:
        """Unit-less cost used when no measurement is available (lower is better)."""
        return _REF_COST[self]


_REF_DESC = {
    RefLinkClass.SYS: "Cross CPU socket",
    RefLinkClass.NODE: "Same CPU socket",
    RefLinkClass.PHB: "Host PCI bridge",
    RefLinkClass.PXB: "Multiple PCI switches",
    RefLinkClass.PIX: "Single PCI switch",
    RefLinkClass.PSB: "Same board",
    RefLinkClass.NV1: "Single NVLink link",
    RefLinkClass.NV2: "Two NVLink links",
    RefLinkClass.NV3: "Three NVLink links",
    RefLinkClass.NV4: "Four NVLink links",
}
# Nominal costs for the reference taxonomy: one NVLink-class link ~ one xGMI link (1.0); bonded
# links divide it; PCIe classes get progressively more expensive as they cross more fabric.
_REF_COST = {
    RefLinkClass.SYS: 8.0,
    RefLinkClass.NODE: 6.0,
    RefLinkClass.PHB: 5.0,
    RefLinkClass.PXB: 4.0,
    RefLinkClass.PIX: 3.0,
    RefLinkClass.PSB: 2.5,
    RefLinkClass.NV1: 1.0,
    RefLinkClass.NV2: 0.5,
    RefLinkClass.NV3: 1.0 / 3.0,
    RefLinkClass.NV4: 0.25,
}


def default_link_cost(lt: LinkType, hops: int = 1) -> float:
    """Cost of a link when the probe has not measured it.

    The numbers are bandwidth ratios against one xGMI link (cost 1.0): two XCPs of the same
    package talk over on-die Infinity Fabric (~4x a link), PCIe Gen5 x16 host staging is ~1/4 of
    an xGMI link and ~1/8 when it also crosses the socket interconnect.
    """
    if lt == LinkType.SELF:
        return 0.0
    if lt == LinkType.INTERNAL:
        return 0.25
    if lt == LinkType.XGMI:
        return float(max(1, hops))
    if lt == LinkType.PCIE:
        return 4.0
    if lt == LinkType.PCIE_SYS:
        return 8.0
    return 16.0


@dataclass
class GPUInfo:
    """One schedulable device (a whole GPU, or one XCP partition of a GPU in CPX/DPX/QPX mode)."""

    index: int  # node-local device index: the ID used in ALIYUN_COM_GPU_GROUP (design.md:231)
    uuid: str = ""
    bdf: str = ""
    numa: int = 0
    render_minor: int = -1  # /dev/dri/renderD<render_minor>
    card: int = -1  # /dev/dri/card<card>
    kfd_node: int = -1  # KFD topology node id (= HSA agent id)
    physical: int = -1  # physical GPU (OAM) this device belongs to; == index for SPX
    partition: str = "SPX"  # compute partition (amdsmi.h:421-432)
    memory_partition: str = "NPS1"
    model: str = "MI355X"
    gfx: str = "gfx950"
    vram_bytes: int = 0
    healthy: bool = True
    xgmi_links_up: int = -1
    cpu_affinity: str = ""  # local_cpulist of the device's PCI function, e.g. "0-47,96-143"
    pcie_link_ratio: float = -1.0  # trained / capable PCIe (speed x width); -1 = unknown
    # RAS signals read by discovery (amdsmi / amdgpu sysfs); -1 = not readable on this node
    xgmi_links_total: int = -1
    ecc_correctable: int = -1
    ecc_uncorrectable: int = -1
    ecc_deferred: int = -1
    bad_pages: int = -1
    bad_page_threshold: int = -1
    # > 1: this device is one of `shares` time slices of GPU `physical` (topology/shares.py): a pod
    # holding j of them holds j/shares of the GPU.  Each slice owns a disjoint 1/shares of the CUs
    # (HSA_CU_MASK, with --share-cu-mask on); HBM is shared, capped cooperatively at the share
    shares: int = 1
    cus: int = -1  # compute units of the physical GPU (KFD simd_count / simd_per_cu); -1 = unknown

    def __post_init__(self) -> None:
        if self.physical < 0:
            self.physical = self.index

    @property
    def render_node(self) -> int:
        """``/dev/dri/renderD<minor>`` of this device; without a discovered one (fake / fixture
        devices) 128 + index, the physical GPU's for a time slice (slices share their GPU's node)."""
        if self.render_minor >= 0:
            return self.render_minor
        return 128 + (self.physical if self.shares > 1 else self.index)

    @property
    def device_id(self) -> str:
        """Device-plugin ``Device.ID``; stable across restarts (the index, as the reference uses)."""
        return str(self.index)


def _numa_distance(raw) -> Optional[Dict[int, List[int]]]:
    if not raw:
        return None
    return {int(k): [int(x) for x in v] for k, v in raw.items()}


def _quantize_bw(bw: np.ndarray) -> np.ndarray:
    """Measured GB/s on the f16 grid the node annotation carries (topology/codec.py): 0.05 %
    resolution, far below probe noise, and the plugin and the extender then derive identical costs."""
    with np.errstate(over="ignore"):
        return bw.astype(np.float16).astype(np.float64)


def _as_matrix(x, n: int, dtype, fill) -> np.ndarray:
    if x is None:
        m = np.full((n, n), fill, dtype=dtype)
    else:
        m = np.array(x, dtype=dtype)
        if m.shape != (n, n):
            raise ValueError(f"matrix shape {m.shape} != ({n},{n})")
    return m


@dataclass
class Topology:
    """Dense pairwise model of one node.

    Matrices are ``n x n`` with the diagonal meaning "self".  ``bw_gbps`` holds measured
    one-direction p2p bandwidth (``nan`` = not measured); ``cost`` is derived by
    :meth:`recompute_cost` unless supplied explicitly (fixtures do that).
    """

    gpus: List[GPUInfo]
    link_type: np.ndarray
    hops: np.ndarray
    weight: Optional[np.ndarray] = None  # amdsmi_topo_get_link_weight
    bw_gbps: Optional[np.ndarray] = None  # measured by the HIP probe
    cost: Optional[np.ndarray] = None
    ref_gbps: float = DEFAULT_REF_GBPS
    node_name: str = ""
    source: str = "unknown"  # amdsmi | sysfs | fake | fixture
    probe: Dict[str, object] = field(default_factory=dict)
    ref_class: Optional[np.ndarray] = None  # optional RefLinkClass matrix (reference fixtures)
    hbm_gbps: Optional[np.ndarray] = None  # per-device self-copy bandwidth (k=1 probe)
    numa_distance: Optional[Dict[int, List[int]]] = None  # NUMA node -> SLIT distances (sysfs)
    # RDMA NICs ({name, bdf, netdev, state, numa, rate_gbps}) and the PCIe class of every GPU-NIC pair
    # ([gpu][nic]: 1 PIX, 2 PXB, 3 PHB, 4 NODE, 5 SYS, 0 unknown — the reference's taxonomy, design.md:31-47)
    nics: Optional[List[Dict[str, object]]] = None
    gpu_nic: Optional[List[List[int]]] = None

    def __post_init__(self) -> None:
        n = len(self.gpus)
        self.link_type = _as_matrix(self.link_type, n, np.int32, int(LinkType.UNKNOWN))
        self.hops = _as_matrix(self.hops, n, np.int32, 1)
        if self.weight is not None:
            self.weight = _as_matrix(self.weight, n, np.float64, 0.0)
        self.bw_gbps = _quantize_bw(_as_matrix(self.bw_gbps, n, np.float64, np.nan))
        if self.ref_class is not None:
            self.ref_class = _as_matrix(self.ref_class, n, np.int32, 0)
        for i in range(n):
            self.link_type[i, i] = int(LinkType.SELF)
            self.hops[i, i] = 0
        if self.cost is None:
            self.recompute_cost()
        else:
            self.cost = _as_matrix(self.cost, n, np.float64, 0.0)
            np.fill_diagonal(self.cost, 0.0)
        self.validate()

    # ------------------------------------------------------------------ basic accessors
    @property
    def n(self) -> int:
        return len(self.gpus)

    @property
    def numa(self) -> np.ndarray:
        return np.array([g.numa for g in self.gpus], dtype=np.int32)

    @property
    def physical(self) -> np.ndarray:
        return np.array([g.physical for g in self.gpus], dtype=np.int32)

    def healthy_mask(self) -> np.ndarray:
        return np.array([g.healthy for g in self.gpus], dtype=bool)

    def validate(self) -> None:
        n = self.n
        if sorted(g.index for g in self.gpus) != list(range(n)):
            raise ValueError("GPU indices must be 0..n-1")
        if not np.array_equal(self.link_type, self.link_type.T):
            raise ValueError("link_type must be symmetric")
        if not np.allclose(self.cost, self.cost.T, equal_nan=True):
            raise ValueError("cost must be symmetric")
        if n and np.any(self.cost[~np.eye(n, dtype=bool)] < 0):
            raise ValueError("cost must be non-negative")

    # ------------------------------------------------------------------ cost model
    def recompute_cost(self) -> np.ndarray:
        """cost[i,j] = ref_gbps / bw(i,j), symmetrised with the *worse* direction.

        Unmeasured pairs fall back to :func:`default_link_cost` of the discovered link class; a
        reference-taxonomy fixture uses its nominal class cost.  A pair whose measured bandwidth is
        far below nominal (degraded link) therefore costs more than its class suggests — this is
        the point of probing rather than trusting the enum (design.md:47 TODO).
        """
        n = self.n
        c = np.zeros((n, n), dtype=np.float64)
        for i in range(n):
            for j in range(n):
                if i == j:
                    continue
                b1, b2 = self.bw_gbps[i, j], self.bw_gbps[j, i]
                meas = [b for b in (b1, b2) if np.isfinite(b) and b > 0]
                if meas:
                    c[i, j] = self.ref_gbps / min(meas)
                elif self.ref_class is not None and self.ref_class[i, j] > 0:
                    c[i, j] = RefLinkClass(int(self.ref_class[i, j])).nominal_cost()
                else:
                    c[i, j] = default_link_cost(LinkType(int(self.link_type[i, j])), int(self.hops[i, j]))
        # quantised to the 1e-6 grid the JSON annotation carries, so the device plugin and the
        # extender (which decodes the annotation) see bit-identical costs and break ties identically
        c = np.round(np.maximum(c, c.T), 6)
        self.cost = c
        return c

    def set_measured_bw(self, bw: np.ndarray, probe_meta: Optional[Dict[str, object]] = None) -> None:
        self.bw_gbps = _quantize_bw(_as_matrix(bw, self.n, np.float64, np.nan))
        if probe_meta:
            # what discovery read from amdsmi is not the probe's to drop (ops/checks.py rates links by it)
            keep = {k: v for k, v in (self.probe or {}).items() if k == "amdsmi_max_bw_mbps"}
            self.probe = {**keep, **dict(probe_meta)}
        self.recompute_cost()

    # ------------------------------------------------------------------ pair views
    def pairs(self) -> Iterable[Tuple[int, int]]:
        """Unordered pairs i<j; with one GPU there are none (design.md:17-19)."""
        for i in range(self.n):
            for j in range(i + 1, self.n):
                yield i, j

    def subset_cost(self, ids: Sequence[int]) -> float:
        """Mean pairwise cost of a device set (0 for |ids| < 2)."""
        ids = list(ids)
        if len(ids) < 2:
            return 0.0
        sub = self.cost[np.ix_(ids, ids)]
        k = len(ids)
        return float(sub.sum() / (k * (k - 1)))

    def groups(self) -> List[np.ndarray]:
        """Hierarchy levels used for packing/anti-fragmentation, innermost first.

        Level 0: physical GPU (meaningful only when partitioned: several XCPs per GPU).
        Level 1: NUMA domain (socket/NPS).
        """
        return [self.physical.copy(), self.numa.copy()]

    # ------------------------------------------------------------------ (de)serialisation
    def to_dict(self) -> Dict[str, object]:
        def m(a):
            if a is None:
                return None
            return [[(None if (isinstance(v, float) and not math.isfinite(v)) else v) for v in row] for row in a.tolist()]

        d = {
            "version": 1,
            "node": self.node_name,
            "source": self.source,
            "ref_gbps": self.ref_gbps,
            "gpus": [asdict(g) for g in self.gpus],
            "link_type": self.link_type.tolist(),
            "hops": self.hops.tolist(),
            "bw_gbps": m(self.bw_gbps),
            "cost": m(np.round(self.cost, 6)),
            "probe": self.probe,
        }
        if self.weight is not None:
            d["weight"] = self.weight.tolist()
        if self.ref_class is not None:
            d["ref_class"] = self.ref_class.tolist()
        if self.hbm_gbps is not None:
            d["hbm_gbps"] = [None if not np.isfinite(v) else float(v) for v in self.hbm_gbps]
        if self.numa_distance:
            d["numa_distance"] = {str(k): list(v) for k, v in self.numa_distance.items()}
        if self.nics:
            d["nics"] = self.nics
            d["gpu_nic"] = self.gpu_nic
        return d

    def nearest_nics(self, ids: Sequence[int]) -> List[str]:
        """Names of the RDMA NICs closest (PCIe class) to each device of ``ids``, active ports first,
        in device order without repeats: what RCCL should use for inter-node traffic of those GPUs."""
        if not self.nics or not self.gpu_nic:
            return []
        out: List[str] = []
        for i in ids:
            row = self.gpu_nic[int(i)] if int(i) < len(self.gpu_nic) else []
            cands = [(c, "ACTIVE" not in str(self.nics[j].get("state", "")).upper(), j) for j, c in enumerate(row) if c > 0]
            if not cands:
                continue
            best = min(cands)
            for c, down, j in sorted(cands):
                if (c, down) != best[:2]:
                    break
                name = str(self.nics[j]["name"])
                if name not in out:
                    out.append(name)
        return out

    def to_json(self, **kw) -> str:
        return json.dumps(self.to_dict(), separators=(",", ":"), **kw)

    def to_wire(self) -> str:
        """Compact v2 JSON for the node annotation (:mod:`.codec`)."""
        from .codec import encode_v2

        return json.dumps(encode_v2(self), separators=(",", ":"))

    @classmethod
    def from_dict(cls, d: Dict[str, object]) -> "Topology":
        if int(d.get("version", 1)) >= 2:
            from .codec import decode_v2

            return decode_v2(d)
        gpus = [GPUInfo(**g) for g in d["gpus"]]

        def m(a):
            if a is None:
                return None
            return np.array([[np.nan if v is None else v for v in row] for row in a], dtype=np.float64)

        hbm = d.get("hbm_gbps")
        return cls(
            gpus=gpus,
            link_type=np.array(d["link_type"], dtype=np.int32),
            hops=np.array(d["hops"], dtype=np.int32),
            weight=None if d.get("weight") is None else np.array(d["weight"], dtype=np.float64),
            bw_gbps=m(d.get("bw_gbps")),
            cost=m(d.get("cost")),
            ref_gbps=float(d.get("ref_gbps", DEFAULT_REF_GBPS)),
            node_name=str(d.get("node", "")),
            source=str(d.get("source", "unknown")),
            probe=dict(d.get("probe") or {}),
            ref_class=None if d.get("ref_class") is None else np.array(d["ref_class"], dtype=np.int32),
            hbm_gbps=None if hbm is None else np.array([np.nan if v is None else v for v in hbm], dtype=np.float64),
            numa_distance=_numa_distance(d.get("numa_distance")),
            nics=d.get("nics") or None,
            gpu_nic=d.get("gpu_nic") or None,
        )

    @classmethod
    def from_json(cls, s: str) -> "Topology":
        return cls.from_dict(json.loads(s))

    # ------------------------------------------------------------------ constructors
    @classmethod
    def full_mesh(
        cls,
        n: int = 8,
        numa_split: int = 2,
        link_gbps: Optional[float] = None,
        noise: float = 0.0,
        seed: int = 0,
        node_name: str = "mi355x-node",
        partitions_per_gpu: int = 1,
        cores_per_socket: int = 48,
    ) -> "Topology":
        """Synthetic 8x MI355X full xGMI mesh (fixture F7) or its CPX variant (F8).

        ``numa_split`` sockets split the GPUs evenly (0-3 / 4-7 on a 2-socket host).  With
        ``partitions_per_gpu > 1`` every physical GPU exposes that many XCP devices; XCPs of the same
        GPU are joined by INTERNAL links.  Each socket has ``cores_per_socket`` cores with SMT
        (socket s: ``s*C..(s+1)*C-1`` plus siblings ``+S*C``), SLIT 10 local / 32 remote.
        """
        sockets = max(1, numa_split)
        total_cores = sockets * cores_per_socket

        def cpulist(sock: int) -> str:
            a = sock * cores_per_socket
            return f"{a}-{a + cores_per_socket - 1},{a + total_cores}-{a + total_cores + cores_per_socket - 1}"

        rng = np.random.default_rng(seed)
        total = n * partitions_per_gpu
        per_numa = max(1, n // max(1, numa_split))
        part_name = {1: "SPX", 2: "DPX", 3: "TPX", 4: "QPX", 8: "CPX"}.get(partitions_per_gpu, "CPX")
        gpus = []
        for d in range(total):
            phys = d // partitions_per_gpu
            gpus.append(
                GPUInfo(
                    index=d,
                    uuid=f"GPU-{phys:04x}-{d % partitions_per_gpu}",
                    bdf=f"0000:{0x05 + 0x10 * phys:02x}:00.{d % partitions_per_gpu}",
                    numa=min(phys // per_numa, max(0, numa_split - 1)),
                    render_minor=128 + d,
                    card=d,
                    kfd_node=d + 2,
                    physical=phys,
                    partition=part_name,
                    vram_bytes=(288 * 10**9) // partitions_per_gpu,
                    xgmi_links_up=n - 1,
                    cpu_affinity=cpulist(min(phys // per_numa, max(0, numa_split - 1))) if cores_per_socket else "",
                    pcie_link_ratio=1.0,
                )
            )
        lt = np.full((total, total), int(LinkType.XGMI), dtype=np.int32)
        hops = np.ones((total, total), dtype=np.int32)
        for i in range(total):
            for j in range(total):
                if gpus[i].physical == gpus[j].physical and i != j:
                    lt[i, j] = int(LinkType.INTERNAL)
                    hops[i, j] = 0
        bw = None
        if link_gbps is not None:
            bw = np.full((total, total), np.nan)
            for i in range(total):
                for j in range(total):
                    if i == j:
                        continue
                    base = link_gbps * (4.0 if lt[i, j] == int(LinkType.INTERNAL) else 1.0)
                    bw[i, j] = base * (1.0 + noise * rng.uniform(-1, 1))
        slit = {s: [10 if s == t else 32 for t in range(sockets)] for s in range(sockets)}
        return cls(gpus=gpus, link_type=lt, hops=hops, bw_gbps=bw, node_name=node_name, source="fake", numa_distance=slit)

    @classmethod
    def from_ref_matrix(
        cls, classes: Sequence[Sequence[str]], numa: Optional[Sequence[int]] = None, node_name: str = "ref-node"
    ) -> "Topology":
        """Build from an ``nvidia-smi topo -m``-style matrix of abbreviations (fixture F1)."""
        n = len(classes)
        rc = np.zeros((n, n), dtype=np.int32)
        lt = np.zeros((n, n), dtype=np.int32)
        for i in range(n):
            for j in range(n):
                if i == j:
                    continue
                c = RefLinkClass[classes[i][j]]
                rc[i, j] = int(c)
                lt[i, j] = int(c.to_link_type())
        numa = list(numa) if numa is not None else [0] * n
        gpus = [GPUInfo(index=i, numa=numa[i], model="ref", gfx="ref") for i in range(n)]
        return cls(gpus=gpus, link_type=lt, hops=np.ones((n, n), dtype=np.int32), ref_class=rc, node_name=node_name, source="fixture")

    # ------------------------------------------------------------------ pretty
    def render(self) -> str:
        """``amd-smi topology``/``nvidia-smi topo -m``-like table."""
        n = self.n
        hdr = "      " + "".join(f"{'GPU' + str(j):>10}" for j in range(n)) + "   NUMA"
        lines = [hdr]
        for i in range(n):
            cells = []
            for j in range(n):
                if i == j:
                    cells.append(f"{'X':>10}")
                else:
                    lt = LinkType(int(self.link_type[i, j]))
                    bw = self.bw_gbps[i, j]
                    tag = lt.abbr if not np.isfinite(bw) else f"{lt.abbr[:4]}{bw:5.0f}"
                    cells.append(f"{tag:>10}")
            lines.append(f"GPU{i:<3}" + "".join(cells) + f"   {self.gpus[i].numa}")
        return "\n".join(lines)
