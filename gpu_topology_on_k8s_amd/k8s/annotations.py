"""Wire contracts carried by Kubernetes objects — kept byte-compatible.

Node annotations (written by the device plugin, read by the extender):
  * ``GPU_<ABBR>_<i>_<j>: <description>`` — one per unordered device pair, ``design.md:76-82``
    (e.g. ``GPU_SYS_0_1: Cross CPU socket``).  On MI355X the abbreviations are the AMD link classes
    (``GPU_XGMI_0_1: xGMI 1 hop``, ``GPU_INTERNAL_0_1``, ``GPU_PCIE_..``, ``GPU_SYS_..``); the
    reference's NVML abbreviations (SYS/NODE/PHB/PXB/PIX/PSB/NV#) are still parsed.
  * ``<prefix>/topology`` — one JSON document with the full model (measured GB/s matrix, cost,
    NUMA, partitions, probe metadata).  This answers the reference's weight TODO (``design.md:47``).

Pod annotations (written by the extender at bind, flipped by the device plugin at Allocate):
  * ``ALIYUN_COM_GPU_GROUP: 0,1,2,3`` — node-local device indices (``design.md:231``)
  * ``ALIYUN_COM_GPU_ASSIGNED: false|true`` (``design.md:227,243``)
  * ``ALIYUN_COM_GPU_ASSUME_TIME: <unix seconds>`` (``design.md:229,245``)
  * ``gpu-id: 0,2`` — the diagram's alias (``imgs/gpu_topology_on_k8s.png`` step 4), read-only.
"""
from __future__ import annotations

import json
import re
import time
from dataclasses import dataclass
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from ..topology.model import LinkType, RefLinkClass, Topology

__all__ = [
    "ANN_GROUP", "ANN_ASSIGNED", "ANN_ASSUME_TIME", "ANN_GPU_ID_ALIAS", "Contract", "PodAssignment",
    "encode_node_annotations", "decode_node_annotations", "pair_annotations", "parse_pair_annotations",
    "parse_group", "format_group", "package_pair_annotations", "annotations_size", "probing_until",
]

ANN_GROUP = "ALIYUN_COM_GPU_GROUP"
ANN_ASSIGNED = "ALIYUN_COM_GPU_ASSIGNED"
ANN_ASSUME_TIME = "ALIYUN_COM_GPU_ASSUME_TIME"
ANN_GPU_ID_ALIAS = "gpu-id"

DEFAULT_PREFIX = "gputopology.amd.com"
DEFAULT_RESOURCE = "amd.com/gpu"
DEFAULT_SLICE_RESOURCE = "amd.com/gpu-slice"  # time slices of a GPU (topology/shares.py): a pool of their own
COMPAT_RESOURCE = "aliyun.com/gpu"  # design.md:86,105 (aliyun.com/gpu-count in the prose/diagram)

_PAIR_RE = re.compile(r"^GPU_([A-Z0-9]+)_(\d+)_(\d+)$")


@dataclass(frozen=True)
class Contract:
    """Names that make up the cluster-state contract (configurable)."""

    resource_name: str = DEFAULT_RESOURCE
    prefix: str = DEFAULT_PREFIX
    #: extended resource a time-sliced node advertises its slices under.  Gaia keeps resource pools
    #: apart (paper p.3 §III.A, "resource pool pollution"): ``resource_name`` always counts whole
    #: GPUs, so a pod's ``amd.com/gpu: 1`` means one GPU on every node, and a sliced node advertises
    #: 0 of them and S x GPUs of this resource instead.
    slice_resource: str = DEFAULT_SLICE_RESOURCE

    @property
    def topology_key(self) -> str:
        return f"{self.prefix}/topology"

    @property
    def probe_time_key(self) -> str:
        return f"{self.prefix}/probe-time"

    @property
    def probing_key(self) -> str:
        """Node annotation set by the device plugin while an idle-time link re-probe owns the node's
        xGMI links: the unix time until which the extender's filter / sort / bind skip the node (a
        pod admitted mid-probe would share the links with the probe, and a crashed plugin's mark
        expires on its own)."""
        return f"{self.prefix}/probing"

    @property
    def ledger_key(self) -> str:
        """Node annotation: the device sets the extenders have bound onto the node and not yet seen
        settle, ``{"gen": N, "a": {"<ns>/<pod>": {"g": [ids], "t": unix time}}}``.  Written in bind with
        the node's resourceVersion as a precondition, so two extender instances (a scheduler leader
        failover, a DaemonSet of extenders) cannot both hand out one node's free devices: the second
        writer gets 409, re-reads and re-decides (extender/scheduler.py)."""
        return f"{self.prefix}/gpu-ledger"

    @property
    def cordon_key(self) -> str:
        """Node annotation set by the operator: GPUs to take out of service without draining the node
        (an RMA, a flaky HBM stack), as device indices or PCI addresses, comma-separated.  Each names
        its whole physical GPU.  The device plugin advertises them Unhealthy (the kubelet stops counting
        them, the extender stops choosing them); pods already on them keep running."""
        return f"{self.prefix}/cordoned-gpus"

    @property
    def numa_key(self) -> str:
        """Pod annotation: NUMA node(s) of the assigned devices (Gaia B6)."""
        return f"{self.prefix}/numa-nodes"

    @property
    def cpuset_key(self) -> str:
        """Pod annotation: recommended cpuset = the assigned devices' local cores (Gaia B6 CPU binding)."""
        return f"{self.prefix}/cpuset"

    @property
    def validated_key(self) -> str:
        """Pod annotation: the RCCL all-reduce that validated the placement before the container
        started (device plugin PreStartContainer): k, peak size, algBW / busBW."""
        return f"{self.prefix}/validated-allreduce"

    @property
    def numa_pref_key(self) -> str:
        """Pod annotation: NUMA node(s) the pod's host threads live on (CPU-affinity tie-break input)."""
        return f"{self.prefix}/numa-preference"

    @property
    def multi_node_key(self) -> str:
        """Pod annotation ``"true"``: the pod is one member of a multi-node job, so its devices should
        cover as many RDMA NIC domains as possible (placement ``w_nic`` term)."""
        return f"{self.prefix}/multi-node"

    @property
    def memory_key(self) -> str:
        """Pod annotation: GPU memory the pod needs on ONE GPU ("96Gi", "100G", bytes), served like a
        fraction: the fewest partitions / time slices of one GPU whose HBM covers it."""
        return f"{self.prefix}/gpu-memory"

    @property
    def fraction_key(self) -> str:
        """Pod annotation: a fraction 0<m<1 of ONE physical GPU, served as ceil(m * partitions) XCPs
        of one package on a CPX/DPX/QPX node (Gaia Fragment, paper Alg. 2)."""
        return f"{self.prefix}/gpu-fraction"

    @property
    def score_key(self) -> str:
        return f"{self.prefix}/placement-score"

    @property
    def label_model(self) -> str:
        """Node label for heterogeneous-cluster quota (Gaia B7)."""
        return f"{self.prefix}/gpu-model"

    @property
    def label_partition(self) -> str:
        return f"{self.prefix}/compute-partition"

    @property
    def partition_request_label(self) -> str:
        """Node label set by the operator: the compute partition mode (SPX/DPX/QPX/CPX) the device
        plugin should put the node's GPUs in, once no pod holds a device (``--partition-control``).
        ``label_partition`` is what the plugin publishes; this is what the operator asks for."""
        return f"{self.prefix}/compute-partition-request"

    @property
    def memory_partition_request_label(self) -> str:
        """Node label set by the operator: the memory partition mode (NPS1/NPS2/NPS4/NPS8) to apply
        with the compute partition request."""
        return f"{self.prefix}/memory-partition-request"

    @property
    def partition_failed_key(self) -> str:
        """Node annotation written by the device plugin when a requested partition change failed:
        ``<compute>/<memory>: <reason>``; the plugin does not retry that request until the label changes."""
        return f"{self.prefix}/partition-change-failed"

    @property
    def label_gfx(self) -> str:
        return f"{self.prefix}/gfx"

    @property
    def time_slices_label(self) -> str:
        """Node label set by the operator: advertise this node's GPUs as that many time slices."""
        return f"{self.prefix}/time-slices"

    @property
    def active_slices_key(self) -> str:
        """Node annotation written by the device plugin: the time slices per GPU it advertises now.
        A restarted plugin keeps this count while pods hold devices (their GROUP annotations and the
        kubelet's checkpoint name devices of this layout) and switches to a changed label only once
        the node is idle."""
        return f"{self.prefix}/time-slices-active"

    @property
    def label_slices(self) -> str:
        """Node label: devices per physical GPU (time slices or XCP partitions; "1" = whole GPUs), so
        fractional pods can select shared nodes with a nodeSelector."""
        return f"{self.prefix}/devices-per-gpu"

    @property
    def pod_model_key(self) -> str:
        """Pod annotation/label selecting a GPU model (pods without it accept any single model)."""
        return f"{self.prefix}/gpu-model"


# ------------------------------------------------------------------------------ node annotations
def _pair_abbr_desc(t: Topology, i: int, j: int) -> Tuple[str, str]:
    if t.ref_class is not None and int(t.ref_class[i, j]) > 0:
        rc = RefLinkClass(int(t.ref_class[i, j]))
        return rc.name, rc.desc
    lt = LinkType(int(t.link_type[i, j]))
    if lt == LinkType.XGMI:
        h = int(t.hops[i, j])
        return lt.abbr, f"xGMI {h} hop" + ("s" if h != 1 else "")
    return lt.abbr, lt.desc


def pair_annotations(t: Topology) -> Dict[str, str]:
    """``GPU_<ABBR>_<i>_<j>`` for every unordered pair (none for a single GPU, design.md:17-19)."""
    out: Dict[str, str] = {}
    for i, j in t.pairs():
        abbr, desc = _pair_abbr_desc(t, i, j)
        out[f"GPU_{abbr}_{i}_{j}"] = desc
    return out


def parse_pair_annotations(ann: Mapping[str, str]) -> Dict[Tuple[int, int], str]:
    """``{(i, j): ABBR}`` from ``GPU_<ABBR>_<i>_<j>`` keys (AMD or reference abbreviations)."""
    out: Dict[Tuple[int, int], str] = {}
    for k in ann:
        m = _PAIR_RE.match(k)
        if m:
            i, j = int(m.group(2)), int(m.group(3))
            out[(min(i, j), max(i, j))] = m.group(1)
    return out


def package_pair_annotations(t: Topology) -> Dict[str, str]:
    """Partitioned (CPX/DPX/QPX) nodes: one ``GPUPKG_<ABBR>_<p>_<q>`` key per pair of *physical*
    GPUs instead of one ``GPU_<ABBR>_<i>_<j>`` per XCP pair (64 XCPs = 2016 keys, ~50 KB of the
    apiserver's 256 KiB per-object annotation budget).  The different prefix keeps readers of the
    reference contract from taking package ids for device ids."""
    first: Dict[int, int] = {}
    for g in t.gpus:
        first.setdefault(g.physical, g.index)
    pk = sorted(first)
    out: Dict[str, str] = {}
    for a in range(len(pk)):
        for b in range(a + 1, len(pk)):
            abbr, desc = _pair_abbr_desc(t, first[pk[a]], first[pk[b]])
            out[f"GPUPKG_{abbr}_{pk[a]}_{pk[b]}"] = desc
    return out


def encode_node_annotations(t: Topology, contract: Contract = Contract(), with_pairs: bool = True) -> Dict[str, str]:
    """Node annotations: the compact v2 model (topology/codec.py) + the reference's pair keys
    (per device on whole-GPU nodes, per physical GPU on partitioned nodes)."""
    ann = {contract.topology_key: t.to_wire()}
    ts = t.probe.get("ts") if t.probe else None
    if ts:
        ann[contract.probe_time_key] = str(int(ts))
    if with_pairs:
        partitioned = len({g.physical for g in t.gpus}) < t.n
        ann.update(package_pair_annotations(t) if partitioned else pair_annotations(t))
    return ann


def probing_until(ann: Mapping[str, str], contract: Contract = Contract()) -> float:
    """Deadline of a node's re-probe mark (``<prefix>/probing``), 0 when absent or malformed."""
    raw = ann.get(contract.probing_key)
    try:
        return float(raw) if raw not in (None, "") else 0.0
    except (TypeError, ValueError):
        return 0.0


def parse_ledger(ann: Mapping[str, str], contract: Contract = Contract()) -> Dict[str, Tuple[Tuple[int, ...], float]]:
    """Entries of a node's allocation ledger (``Contract.ledger_key``): pod key -> (device ids, unix
    time of the bind).  A malformed ledger reads as empty (the next bind rewrites it)."""
    raw = ann.get(contract.ledger_key)
    if not raw:
        return {}
    try:
        d = json.loads(raw)
        return {str(k): (tuple(int(i) for i in v["g"]), float(v["t"])) for k, v in (d.get("a") or {}).items()}
    except (ValueError, TypeError, KeyError, AttributeError):
        return {}


def ledger_gen(ann: Mapping[str, str], contract: Contract = Contract()) -> int:
    try:
        return int(json.loads(ann.get(contract.ledger_key) or "{}").get("gen", 0))
    except (ValueError, TypeError, AttributeError):
        return 0


def ledger_uids(ann: Mapping[str, str], contract: Contract = Contract()) -> Dict[str, str]:
    """Pod UID of each ledger entry that records one (``"u"``; entries of round-5 writers have none)."""
    try:
        d = json.loads(ann.get(contract.ledger_key) or "{}")
        return {str(k): str(v["u"]) for k, v in (d.get("a") or {}).items() if isinstance(v, dict) and v.get("u")}
    except (ValueError, TypeError, AttributeError):
        return {}


def dump_ledger(entries: Mapping[str, Tuple[Sequence[int], float]], gen: int, uids: Optional[Mapping[str, str]] = None) -> str:
    """The ledger annotation's value; ``uids`` adds each entry's pod UID (an entry of a re-created pod
    of the same name is then told apart from its predecessor's)."""
    uids = uids or {}
    return json.dumps({"gen": int(gen), "a": {k: {"g": [int(i) for i in g], "t": round(float(t), 3),
                                                  **({"u": uids[k]} if uids.get(k) else {})}
                                               for k, (g, t) in sorted(entries.items())}}, separators=(",", ":"))


def annotations_size(ann: Mapping[str, str]) -> int:
    """Bytes the apiserver counts against its 256 KiB per-object annotation limit (keys + values)."""
    return sum(len(k.encode()) + len(v.encode()) for k, v in ann.items())


def topology_from_pairs(pairs: Dict[Tuple[int, int], str], n: Optional[int] = None) -> Topology:
    """Rebuild a class-only model from pair annotations alone (a node written by a reference plugin)."""
    if n is None:
        n = 1 + max([max(p) for p in pairs] or [0])
    abbrs = {a.name for a in RefLinkClass}
    if pairs and all(v in abbrs for v in pairs.values()):
        m = [["PHB"] * n for _ in range(n)]
        for (i, j), a in pairs.items():
            m[i][j] = m[j][i] = a
        return Topology.from_ref_matrix(m, node_name="")
    from ..topology.model import GPUInfo

    lt = np.full((n, n), int(LinkType.UNKNOWN), dtype=np.int32)
    for (i, j), a in pairs.items():
        try:
            v = int(LinkType.from_abbr(a))
        except KeyError:
            v = int(LinkType.UNKNOWN)
        lt[i, j] = lt[j, i] = v
    return Topology(gpus=[GPUInfo(index=i) for i in range(n)], link_type=lt, hops=np.ones((n, n), dtype=np.int32), source="pair-annotations")


def decode_node_annotations(ann: Mapping[str, str], contract: Contract = Contract(), node_name: str = "") -> Optional[Topology]:
    """Topology from a node's annotations: the JSON model if present, else the pair annotations."""
    raw = ann.get(contract.topology_key)
    if raw:
        t = Topology.from_json(raw)
        if node_name:
            t.node_name = node_name
        return t
    pairs = parse_pair_annotations(ann)
    if pairs:
        t = topology_from_pairs(pairs)
        t.node_name = node_name
        return t
    return None


# ------------------------------------------------------------------------------- pod annotations
def parse_group(s: Optional[str]) -> Optional[List[int]]:
    if s is None:
        return None
    s = s.strip()
    if not s:
        return []
    return [int(x) for x in s.split(",") if x.strip() != ""]


def format_group(ids: Sequence[int]) -> str:
    return ",".join(str(int(i)) for i in ids)


@dataclass
class PodAssignment:
    """The allocation state a pod carries in its annotations."""

    group: List[int]
    assigned: bool
    assume_time: int

    @classmethod
    def from_annotations(cls, ann: Optional[Mapping[str, str]]) -> Optional["PodAssignment"]:
        """The assignment a pod carries, or None.  A GROUP that is not a list of device indices
        ("a,b", "-1", a non-string) is no assignment: any user can annotate their own pod, and one such
        pod must not stop the extender from reading its node or the plugin from admitting pods (the pod
        then counts by its resource request, like any pod without a GROUP)."""
        ann = ann if isinstance(ann, Mapping) else {}
        try:
            g = parse_group(ann.get(ANN_GROUP))
            if g is None:
                g = parse_group(ann.get(ANN_GPU_ID_ALIAS))  # diagram alias, read-only
        except (ValueError, AttributeError, TypeError):
            return None
        if g is None or any(i < 0 for i in g):
            return None
        assigned = str(ann.get(ANN_ASSIGNED, "false")).lower() == "true"
        try:
            at = int(ann.get(ANN_ASSUME_TIME, "0"))
        except ValueError:
            at = 0
        return cls(group=g, assigned=assigned, assume_time=at)

    def to_annotations(self) -> Dict[str, str]:
        return {
            ANN_GROUP: format_group(self.group),
            ANN_ASSIGNED: "true" if self.assigned else "false",
            ANN_ASSUME_TIME: str(int(self.assume_time)),
        }

    @classmethod
    def assumed(cls, ids: Sequence[int], now: Optional[float] = None) -> "PodAssignment":
        return cls(group=list(ids), assigned=False, assume_time=int(now if now is not None else time.time()))


def dumps_compact(obj) -> str:
    return json.dumps(obj, separators=(",", ":"))
