"""One identity per device: topology index <-> PCI BDF <-> HIP ordinal.

Reference: ``design.md:239`` hands the chosen device list to the container (``NVIDIA_VISIBLE_DEVICES``,
which the NVIDIA runtime resolves by index *on the host*).  On ROCm the container only gets the
``/dev/dri/renderD*`` nodes of its devices (``deviceplugin/plugin.py`` Allocate) and HIP renumbers
what it can open as ordinals ``0..k-1``, so a node-local index from ``ALIYUN_COM_GPU_GROUP`` (say
``4,5,6,7``) is *not* a HIP ordinal inside the pod, and under ``HIP_VISIBLE_DEVICES`` it is not one
on the host either.  The stable key is the PCI address: amdsmi/KFD give it per topology index
(``GPUInfo.bdf``), ``hipDeviceGetPCIBusId`` gives it per HIP ordinal, and the device plugin passes
it into the container (``GTK_GPU_BDFS``).  Everything that turns a topology index into a device to
run on (``gtk validate``, the link probe, ``choose_subset``/``bench.py``) goes through
:class:`DeviceMap`.

XCP partitions (CPX/DPX/QPX) of one GPU may report the same bus/device with different functions or,
on some drivers, the very same BDF; equal BDFs are matched in order on both sides (both enumerate a
package's partitions in XCP order).
"""
from __future__ import annotations

import logging
import os
import re
from typing import Dict, List, Optional, Sequence

log = logging.getLogger(__name__)

__all__ = ["normalize_bdf", "hip_device_bdfs", "DeviceMap", "resolve_group", "ENV_GROUP", "ENV_BDFS", "ENV_FRACTION",
           "ENV_SLICES", "fractions_from_env"]

#: container env written by Allocate: node-local indices (GROUP order) and their PCI addresses
ENV_GROUP = "GTK_GPU_GROUP"
ENV_BDFS = "GTK_GPU_BDFS"
#: on a time-sliced node (topology/shares.py): the share of each GROUP GPU the pod holds, and the
#: slice ids the kubelet allocated (GROUP then names the physical GPUs behind them)
ENV_FRACTION = "GTK_GPU_FRACTION"
ENV_SLICES = "GTK_GPU_SLICES"

_BDF_RE = re.compile(r"^(?:([0-9a-fA-F]{1,8}):)?([0-9a-fA-F]{1,2}):([0-9a-fA-F]{1,2})\.([0-7])$")


def normalize_bdf(s: str) -> str:
    """``dddd:bb:dd.f`` in lower-case hex ('' for anything unparseable).  Accepts a missing domain
    (``05:00.0``), upper case (``0000:05:00.0`` from HIP) and amdsmi's 4-digit domain."""
    m = _BDF_RE.match((s or "").strip())
    if not m:
        return ""
    dom, bus, dev, fn = m.groups()
    return f"{int(dom or '0', 16):04x}:{int(bus, 16):02x}:{int(dev, 16):02x}.{int(fn)}"


def hip_device_bdfs() -> List[str]:
    """PCI address of every HIP ordinal this process can see (``hipDeviceGetPCIBusId`` through the
    native probe module); ``[]`` without a GPU runtime."""
    from .._native import NativeUnavailable, load

    try:
        p = load("_probe")
    except NativeUnavailable:
        return []
    n = int(p.device_count())
    return [normalize_bdf(str(p.device_props(i)["pci_bus_id"])) for i in range(n)]


class DeviceMap:
    """Bijection between the topology indices this process can reach and its HIP ordinals.

    ``by_bdf`` is True when the PCI addresses decided the mapping.  Without any BDF match (fake or
    fixture topologies, whose addresses are synthetic) the map is the identity over
    ``min(n_topology, n_visible)`` devices and ``by_bdf`` is False, which callers report.
    """

    def __init__(self, hip_of_index: Dict[int, int], n_topology: int, n_visible: int, by_bdf: bool):
        self.hip_of_index = dict(hip_of_index)
        self.index_of_hip = {h: i for i, h in self.hip_of_index.items()}
        self.n_topology = n_topology
        self.n_visible = n_visible
        self.by_bdf = by_bdf

    # ------------------------------------------------------------------ construction
    @classmethod
    def match(cls, topo_bdfs: Sequence[str], visible_bdfs: Sequence[str]) -> "DeviceMap":
        tb = [normalize_bdf(b) for b in topo_bdfs]
        vb = [normalize_bdf(b) for b in visible_bdfs]
        queues: Dict[str, List[int]] = {}
        for i, b in enumerate(tb):
            if b:
                queues.setdefault(b, []).append(i)
        out: Dict[int, int] = {}
        for h, b in enumerate(vb):
            q = queues.get(b)
            if b and q:
                out[q.pop(0)] = h
        if out:
            missing = [h for h in range(len(vb)) if h not in set(out.values())]
            if missing:
                log.warning("HIP ordinals %s have no device in the topology (BDFs %s)", missing, [vb[h] for h in missing])
            return cls(out, len(tb), len(vb), True)
        n = min(len(tb), len(vb))
        return cls({i: i for i in range(n)}, len(tb), len(vb), False)

    @classmethod
    def for_topology(cls, topo, visible_bdfs: Optional[Sequence[str]] = None) -> "DeviceMap":
        """Map ``topo`` onto this process's HIP devices (queried when ``visible_bdfs`` is None)."""
        vis = hip_device_bdfs() if visible_bdfs is None else list(visible_bdfs)
        return cls.match([g.bdf for g in topo.gpus], vis)

    @classmethod
    def identity(cls, n: int) -> "DeviceMap":
        return cls({i: i for i in range(n)}, n, n, False)

    # ------------------------------------------------------------------ queries
    def hip(self, index: int) -> int:
        try:
            return self.hip_of_index[int(index)]
        except KeyError:
            raise KeyError(f"topology device {index} is not visible to HIP in this process "
                           f"(visible topology indices: {self.visible_indices()})") from None

    def index(self, hip: int) -> int:
        return self.index_of_hip[int(hip)]

    def visible_indices(self) -> List[int]:
        return sorted(self.hip_of_index)

    def hidden_indices(self) -> List[int]:
        return [i for i in range(self.n_topology) if i not in self.hip_of_index]

    @property
    def complete(self) -> bool:
        """Every HIP ordinal is a known topology device."""
        return len(self.hip_of_index) == self.n_visible

    def to_dict(self) -> Dict[str, object]:
        return {"by_bdf": self.by_bdf, "hip_of_index": {str(i): h for i, h in sorted(self.hip_of_index.items())}}


def resolve_group(group: Sequence[int], *, bdfs: Optional[Sequence[str]] = None, topology=None,
                  visible_bdfs: Optional[Sequence[str]] = None) -> List[int]:
    """HIP ordinals of the node-local devices ``group`` (a pod's ``ALIYUN_COM_GPU_GROUP``).

    Resolution, first that applies:
      1. ``bdfs`` (``GTK_GPU_BDFS`` from Allocate, same order as ``group``) matched against the
         visible devices' PCI addresses;
      2. ``topology`` (the node model, e.g. ``gtk topo --output json``): GROUP index -> its BDF -> HIP;
      3. a container that sees exactly ``len(group)`` devices: HIP keeps PCI order and GROUP indices
         follow the node's HIP order, so the sorted GROUP maps monotonically onto ``0..k-1``;
      4. otherwise the indices are taken as ordinals when all of them exist (a host-level run).
    Raises ``ValueError`` when the group cannot be placed on the visible devices.
    """
    group = [int(g) for g in group]
    vis = hip_device_bdfs() if visible_bdfs is None else [normalize_bdf(b) for b in visible_bdfs]
    if bdfs:
        want = [normalize_bdf(b) for b in bdfs]
        if len(want) != len(group):
            raise ValueError(f"{ENV_BDFS} has {len(want)} entries for a group of {len(group)}")
        m = DeviceMap.match(want, vis)
        if m.by_bdf and len(m.hip_of_index) == len(group):
            return [m.hip(i) for i in range(len(group))]
        raise ValueError(f"devices {want} are not all visible (visible: {vis})")
    if topology is not None:
        m = DeviceMap.for_topology(topology, vis)
        if m.by_bdf:
            return [m.hip(g) for g in group]
    n = len(vis)
    if n == len(group):
        order = sorted(range(len(group)), key=lambda p: group[p])
        out = [0] * len(group)
        for rank, pos in enumerate(order):
            out[pos] = rank
        return out
    if all(0 <= g < n for g in group):
        return list(group)
    raise ValueError(f"group {group} cannot be mapped onto {n} visible devices without {ENV_BDFS} or a topology")


def group_from_env(env: Optional[Dict[str, str]] = None):
    """(group, bdfs) from the container environment Allocate wrote (empty lists when unset)."""
    env = os.environ if env is None else env
    g = [int(x) for x in env.get(ENV_GROUP, "").split(",") if x.strip()]
    b = [x.strip() for x in env.get(ENV_BDFS, "").split(",") if x.strip()]
    return g, b


def fractions_from_env(env: Optional[Dict[str, str]] = None) -> List[float]:
    """The pod's share of each GROUP GPU (``GTK_GPU_FRACTION``; empty when it holds whole GPUs)."""
    env = os.environ if env is None else env
    return [float(x) for x in env.get(ENV_FRACTION, "").split(",") if x.strip()]
