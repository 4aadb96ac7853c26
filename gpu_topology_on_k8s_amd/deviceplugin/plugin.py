"""kubelet device plugin advertising the MI355X devices of one node.

Reference behaviour:
  * ``design.md:57-82`` — at init, read the GPU-pair topology and publish it as node annotations
    ``GPU_<ABBR>_<i>_<j>``.  Here the node additionally gets one JSON annotation with the measured
    cost model and labels for the GPU model / partition mode (heterogeneous quota, Gaia B7).
  * ``design.md:84-86`` — advertise the extended resource through ``ListAndWatch``.  Each device is
    reported with its NUMA node (``TopologyInfo``) and live health.
  * ``design.md:236-246`` — ``Allocate`` finds the pod the devices belong to through the pod
    annotations, injects the devices and flips ``ALIYUN_COM_GPU_ASSIGNED=true`` with a fresh
    ``ALIYUN_COM_GPU_ASSUME_TIME``.  Instead of ``NVIDIA_VISIBLE_DEVICES`` for nvidia-docker, the
    container gets the ROCm device nodes: ``/dev/kfd`` plus ``/dev/dri/renderD<minor>`` (and
    ``card<N>``) of each allocated device — plain containerd, no runtime hook.
  * ``GetPreferredAllocation`` (kubelet API, not in the 2019 design) returns the extender's GROUP so
    the kubelet allocates exactly the annotated devices; without an annotated pod it runs the
    placement core itself.

Pod <-> Allocate association (the kubelet does not say which pod it is allocating for, SURVEY §7.3
#4).  The kubelet's device manager calls ``GetPreferredAllocation`` and ``Allocate`` once per
container, with that container's count, init containers first, and hands a regular init container's
devices on to the containers after it.  A pending pod's containers (its spec) say which count its
next call asks for, so a request of ``n`` devices is matched to the pod whose next container asks
``n``: a pod whose admission is under way first, then the oldest ``ASSUME_TIME`` (the design's
implicit scheme).  ``GetPreferredAllocation`` answers with the part of that pod's GROUP the container
should get; ``Allocate`` records the devices against the GROUP and flips ``ASSIGNED=true`` once the
whole GROUP has been allocated.  Devices outside the GROUP rewrite it to the kubelet's choice.  A pod
scheduled around the extender (no GROUP) is annotated with what the kubelet gave its containers, so
the extender sees the usage.
"""
from __future__ import annotations

import contextlib
import itertools
import json
import logging
import math
import os
import threading
import time
from concurrent import futures
from typing import Callable, Dict, List, Optional, Sequence, Set, Tuple

import grpc
import numpy as np

from ..k8s.annotations import (ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GROUP, Contract, PodAssignment, decode_node_annotations,
                               encode_node_annotations, format_group)
from ..k8s.api import Conflict, KubeAPI
from ..k8s.events import record_event
from ..k8s.objects import annotations as obj_annotations
from ..k8s.objects import meta, pod_device_steps, pod_gpu_request, pod_is_terminal, pod_key, pod_phase
from ..placement import NoFeasiblePlacement, PlacementPolicy
from ..placement.core import select_with
from ..placement.numa_align import TopologyManager, tm_labels
from ..topology.cpus import recommended_cpuset
from ..topology.identity import ENV_BDFS, ENV_FRACTION, ENV_GROUP, ENV_SLICES
from ..topology.model import Topology
from ..topology.shares import cu_mask_env, format_cus, physical_group, share_cus, share_fractions, slices_per_gpu
from . import proto as pb
from .podresources import POD_RESOURCES_SOCKET, list_pod_resources
from .metrics import PluginMetrics

log = logging.getLogger(__name__)

__all__ = ["DevicePluginServer", "PluginConfig", "placeholder_dev_tree", "node_is_idle", "startup_topology"]

#: pod annotation whose ``KEY=VALUE`` lines are passed into the container (RCCL / NCCL tuning only)
RCCL_ENV_ANNOTATION_SUFFIX = "rccl-env"
_ENV_PREFIXES = ("NCCL_", "RCCL_", "HSA_", "HIP_", "GPU_MAX_HW_QUEUES")


def node_is_idle(api: KubeAPI, node_name: str, resource_names: Sequence[str]) -> bool:
    """True when no live pod on ``node_name`` holds a device: neither an annotated GROUP (assumed or
    allocated) nor a device request scheduled around the extender.  Any API error counts as busy."""
    try:
        pods = [p for p in api.list_pods(node_name=node_name) if not pod_is_terminal(p)]
    except Exception as e:
        log.warning("listing pods on %s failed: %s", node_name, e)
        return False
    for p in pods:
        if PodAssignment.from_annotations(obj_annotations(p)) is not None:
            return False
        try:
            if pod_gpu_request(p, resource_names) > 0:
                return False
        except ValueError:
            return False
    return True


def startup_topology(discovered: Topology, api: Optional[KubeAPI], node_name: str, contract: Contract,
                     resource_names: Sequence[str], probe_fn: Optional[Callable[[], Optional[Topology]]]) -> Tuple[Topology, str]:
    """The topology a (re)starting plugin publishes, and how it was obtained.

    A plugin restart or upgrade on a node running jobs must not saturate every xGMI link under live
    training (and publish contention-skewed costs): while any pod holds a device the measured matrix
    already on the node annotation is carried over onto the fresh discovery (same devices, same PCI
    addresses) and no probe runs.  The probe runs only on an idle node (or with no apiserver at all,
    where the operator's ``--probe`` is the only signal)."""
    if probe_fn is None:
        return discovered, "probe off"
    if api is not None and node_name and not node_is_idle(api, node_name, resource_names):
        prev = None
        try:
            prev = decode_node_annotations(obj_annotations(api.get_node(node_name)), contract, node_name=node_name)
        except Exception as e:  # noqa: BLE001 - unreadable annotation: nothing to reuse
            log.warning("reading the published topology of %s failed: %s", node_name, e)
        measured = prev is not None and ((prev.bw_gbps is not None and np.isfinite(prev.bw_gbps).any())
                                         or (prev.hbm_gbps is not None and np.isfinite(prev.hbm_gbps).any()))
        if measured and prev.n == discovered.n and [g.bdf for g in prev.gpus] == [g.bdf for g in discovered.gpus]:
            discovered.hbm_gbps = prev.hbm_gbps
            discovered.set_measured_bw(prev.bw_gbps, dict(prev.probe, reused=True))
            return discovered, "reused the published matrix (devices in use: probe skipped)"
        return discovered, "devices in use and no compatible published matrix: probe skipped, link classes only"
    probed = probe_fn()
    if probed is not None and probed.n == discovered.n:
        probed.node_name = discovered.node_name
        return probed, "probed"
    return discovered, "probe unavailable: link classes only"


def placeholder_dev_tree(root: str, topo: Topology) -> str:
    """Create empty stand-ins for ``kfd`` and every device's ``dri/renderD*`` / ``dri/card*`` under
    ``root`` (the ``--dev-root`` of a kind node or the cluster simulation, where no real ROCm device
    nodes exist but the Allocate -> container path must still be exercised end to end)."""
    os.makedirs(os.path.join(root, "dri"), exist_ok=True)
    names = ["kfd"]
    for g in topo.gpus:
        names.append(f"dri/renderD{g.render_node}")
        if g.card >= 0:
            names.append(f"dri/card{g.card}")
    for n in names:
        open(os.path.join(root, n), "a").close()
    return root


class PluginConfig:
    def __init__(self, resource_name: str = "amd.com/gpu", socket_dir: str = pb.DEVICE_PLUGIN_PATH,
                 socket_name: str = "amd-gpu-topology.sock", kubelet_socket: Optional[str] = None, dev_root: str = "/dev",
                 node_name: str = "", contract: Optional[Contract] = None, health_interval: float = 5.0,
                 publish_node: bool = True, pass_rccl_env: bool = True, policy: PlacementPolicy = PlacementPolicy(),
                 resource_aliases: Sequence[str] = ("aliyun.com/gpu", "aliyun.com/gpu-count"),
                 reprobe_interval: float = 0.0, reprobe_tolerance: float = 0.15, device_specs: str = "strict",
                 prestart_validate: bool = False, validate_timeout: float = 120.0,
                 pod_resources_socket: Optional[str] = POD_RESOURCES_SOCKET, reconcile_interval: float = 10.0,
                 cdi_dir: str = "/var/run/cdi", cdi_kind: str = "amd.com/gpu", nic_env: bool = True,
                 share_cu_mask: bool = True, probe_mark_s: float = 300.0, probe_settle_s: float = 2.0,
                 probe_yield_s: float = 20.0, share_guard: str = "off", guard_dir: str = "/var/lib/gtk-vgpu",
                 guard_lib: Optional[str] = None, admission_settle_s: float = 5.0,
                 topology_manager: Optional[TopologyManager] = None, container_ipc_mode: Optional[str] = None):
        self.resource_name = resource_name
        # HSA_ENABLE_IPC_MODE_LEGACY handed to every allocated container (None: the plugin's own value;
        # "": none).  On hosts whose amdgpu driver exports IPC handles only as dma-bufs, ROCr needs 0 or a
        # multi-process RCCL job in the pod fails in hipIpcGetMemHandle (docs/OPERATIONS.md "IPC")
        self.container_ipc_mode = (os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "") if container_ipc_mode is None
                                   else container_ipc_mode)
        self.socket_dir = socket_dir
        self.socket_name = socket_name
        self.kubelet_socket = kubelet_socket or os.path.join(socket_dir, "kubelet.sock")
        self.dev_root = dev_root
        self.node_name = node_name
        self.contract = contract or Contract(resource_name=resource_name)
        self.health_interval = health_interval
        self.publish_node = publish_node
        self.pass_rccl_env = pass_rccl_env
        self.policy = policy
        self.resource_aliases = tuple(resource_aliases)
        # re-measure the links every `reprobe_interval` s while no pod holds a device (0 = never);
        # republish when any measured pair moved by more than `reprobe_tolerance` (relative)
        self.reprobe_interval = reprobe_interval
        self.reprobe_tolerance = reprobe_tolerance
        # a re-probe marks the node `<prefix>/probing` for at most `probe_mark_s` (the extender skips
        # it), waits `probe_settle_s` for binds already in flight, and an Allocate arriving mid-probe
        # waits at most `probe_yield_s` for the cancelled probe to release the GPUs
        self.probe_mark_s = probe_mark_s
        self.probe_settle_s = probe_settle_s
        self.probe_yield_s = probe_yield_s
        # Allocate's DeviceSpecs: "strict" = /dev/kfd + every device's render/card node, Allocate fails
        # if one is missing on the node (a container must never start without its GPU); "stub" = only
        # the nodes that exist under dev_root (a kind node with fake GPUs has none: envs + annotations
        # only, BASELINE config 1); "cdi" = CDI names (``cdi_kind=<index>``) resolved by the spec the
        # plugin writes into ``cdi_dir`` (deviceplugin/cdi.py): the runtime injects the nodes
        if device_specs not in ("strict", "stub", "cdi"):
            raise ValueError(f"device_specs must be strict|stub|cdi, got {device_specs!r}")
        self.device_specs = device_specs
        self.cdi_dir = cdi_dir
        self.cdi_kind = cdi_kind
        # multi-node RCCL: NCCL_IB_HCA = the RDMA NICs behind the allocated GPUs' own PCIe switches
        # (Topology.nearest_nics); a pod's RCCL env annotation still overrides it
        self.nic_env = nic_env
        # time-sliced nodes (topology/shares.py): confine a pod holding part of a GPU to its slices'
        # compute units (HSA_CU_MASK); off = slices share every CU (temporal sharing only)
        self.share_cu_mask = share_cu_mask
        # the container-side tier of a time-sliced share (csrc/vgpu/vgpu_guard.cpp, Gaia's two-tier
        # vGPU): a pod holding part of a GPU gets libgtk_vgpu.so mounted and preloaded, which caps its
        # HIP allocations at the share's HBM and forces its HSA_CU_MASK.  "env" = LD_PRELOAD in the
        # container env; "preload" = also an /etc/ld.so.preload mount (survives an env override);
        # "off" = cooperative only.  `guard_dir` is a host directory the plugin writes the library and
        # the per-allocation configs to (a hostPath mounted at the same path into the DaemonSet)
        if share_guard not in ("off", "env", "preload"):
            raise ValueError(f"share_guard must be off|env|preload, got {share_guard!r}")
        self.share_guard = share_guard
        self.guard_dir = guard_dir
        self.guard_lib = guard_lib
        # flow step 8: before the container starts, an RCCL all-reduce over exactly
        # the allocated devices (kubelet PreStartContainer) validates the placement; the measured
        # bus bandwidth is recorded on the pod
        self.prestart_validate = prestart_validate
        self.validate_timeout = validate_timeout
        # Allocate has no pod identity: two same-size pods assumed on one node can be admitted in the
        # other order, leaving their GROUP annotations swapped.  Every `reconcile_interval` s the
        # annotations are corrected to the kubelet's pod-resources API (None / "" = off)
        self.pod_resources_socket = pod_resources_socket or ""
        self.reconcile_interval = reconcile_interval
        # the kubelet allocates a pod container by container, back to back: a Pending pod is reconciled
        # only once no Allocate has come for this long (its calls may still be under way)
        self.admission_settle_s = admission_settle_s
        # the kubelet's Topology Manager, published as node labels so the extender picks the devices the
        # kubelet will offer (placement/numa_align.py)
        self.topology_manager = topology_manager or TopologyManager()

    @property
    def socket_path(self) -> str:
        return os.path.join(self.socket_dir, self.socket_name)


class _Admission:
    """A pod the kubelet is admitting: it calls ``Allocate`` once per container, so a
    GROUP is claimed over several calls.  In memory only, while the pod is Pending."""

    __slots__ = ("key", "uid", "claimed", "done")

    def __init__(self, key: str, uid: str) -> None:
        self.key, self.uid = key, uid
        self.claimed: set = set()  # devices its containers got so far
        self.done = 0  # its Allocate calls so far (containers requesting devices, kubelet order)


class _Candidate:
    """A pending pod an ``Allocate`` / ``GetPreferredAllocation`` may be for."""

    __slots__ = ("pod", "key", "pa", "steps", "adm")

    def __init__(self, pod: dict, key: str, pa: Optional[PodAssignment], steps: List[Tuple[str, int, str]],
                 adm: Optional[_Admission]) -> None:
        self.pod, self.key, self.pa, self.steps, self.adm = pod, key, pa, steps, adm

    def next_size(self) -> Optional[int]:
        """Devices the pod's next container asks for (None: not known from its spec, or all done)."""
        done = self.adm.done if self.adm is not None else 0
        return self.steps[done][1] if done < len(self.steps) else None


class AllocationHold:
    """State shared by a partition switch and the Allocate calls it holds (``allocation_hold``)."""

    def __init__(self) -> None:
        self.waiters = 0  # Allocate calls waiting for the switch
        self.started = False  # the switch passed its last idle check and runs amdsmi steps
        self.switched = False  # ... and changed the package's modes

    def contended(self) -> bool:
        return self.waiters > 0


class DevicePluginServer:
    def __init__(self, topology: Topology, config: Optional[PluginConfig] = None, api: Optional[KubeAPI] = None,
                 health_fn: Optional[Callable[[Topology], Dict[int, bool]]] = None, clock: Callable[[], float] = time.time,
                 reprobe_fn: Optional[Callable[[], Optional[Topology]]] = None,
                 validate_fn: Optional[Callable[[Sequence[int]], Dict[str, object]]] = None):
        self.cfg = config or PluginConfig()
        self.validate_fn = validate_fn or self._validate_in_child
        self.topology = topology
        self.api = api
        self.health_fn = health_fn
        self.reprobe_fn = reprobe_fn
        self.reprobes = 0  # completed re-measurements
        self.republished = 0  # ... of which changed the published matrix
        self.clock = clock
        self._health: Dict[int, bool] = {g.index: bool(g.healthy) for g in topology.gpus}
        self._cond = threading.Condition()
        self._version = 0
        self._server: Optional[grpc.Server] = None
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self._alloc_lock = threading.Lock()
        self._alloc_cond = threading.Condition(self._alloc_lock)  # Allocate waits here for a probe to yield
        # one maintenance operation on the GPUs at a time: an idle-time re-probe (a HIP child on every
        # GPU) and a partition switch (deviceplugin/repartition.py) must never overlap
        self.maintenance = threading.Lock()
        self._probing = False  # set (under _alloc_lock) while an idle-time re-probe owns the links
        self._cancel = threading.Event()  # set by an Allocate arriving mid-probe: the probe stops
        self._guard_seq = itertools.count(1)  # unique per-allocation guard files (_guard_files)
        self._hold: Optional["AllocationHold"] = None  # a partition switch holds Allocate (allocation_hold)
        self._stale_layout = ""  # set when a switch changed the device layout: Allocate refuses until the restart
        self._guard_ready = False  # install_guard() put libgtk_vgpu.so into cfg.guard_dir
        self.allocations: List[Tuple[str, Tuple[int, ...]]] = []  # (pod key or "", ids) log
        self._admissions: Dict[str, _Admission] = {}  # pod key -> admission in progress (under _alloc_lock)
        # admission units: the devices of consecutive Allocate calls linked by reuse (an init container's
        # devices handed on), i.e. of one kubelet pod admission whichever pod the calls were matched to
        self._unit_of: Dict[int, set] = {}  # device -> its unit (from the latest call that allocated it)
        self._chain: Optional[Tuple[set, Optional[_Admission]]] = None  # the previous call's unit and record
        self._last_alloc = -1e9  # monotonic time the last Allocate ended
        self._claimed_by: Optional[_Admission] = None  # the record _claim_pod matched the current call to
        # must_include of the GetPreferredAllocation calls since the last Allocate (None: there was none).
        # The kubelet asks before every container whose reused devices do not cover its request, with
        # must_include = the reused devices, and skips the call only when they cover it: so this tells
        # which devices of the next Allocate are reused (all of them when None)
        self._gpa_must: Optional[set] = None
        self.registered = 0
        self.metrics = PluginMetrics()
        self.metrics.set_topology(topology)
        # set when re-discovery finds a different device set (partition switch, hot removal): the
        # daemon exits for a clean restart instead of advertising stale device IDs
        self.layout_change = threading.Event()
        self.layout_change_reason = ""
        # devices held Unhealthy by a GPU event (reset in progress) whatever the RAS poll says
        self._holds: Dict[int, str] = {}
        # devices the operator's cordon annotation names (held with CORDON_HOLD unless a reset holds them)
        self._cordon_want: Set[int] = set()
        self._cordon_unknown: List[str] = []
        self._reprobe_now = threading.Event()  # a GPU reset finished: re-measure as soon as the node is idle
        self.event_source = None  # deviceplugin.events.GpuEventWatcher (amdsmi event notification)
        # liveness (/healthz): the monitor loop's last pass, and since when re-registration has failed
        self._monitor_beat: Optional[float] = None
        self._register_failing_since: Optional[float] = None
        self._started = False
        self._register_required = True

    # ------------------------------------------------------------------ device view
    def devices(self) -> List[pb.Device]:
        out = []
        for g in self.topology.gpus:
            d = pb.Device(ID=g.device_id, health=pb.HEALTHY if self._health.get(g.index, True) else pb.UNHEALTHY)
            d.topology.nodes.add(ID=int(g.numa))
            out.append(d)
        return out

    def set_health(self, index: int, healthy: bool) -> None:
        """Fault injection / health monitor entry: re-advertise through every ListAndWatch stream."""
        self.set_health_many({index: healthy})

    def set_health_many(self, states: Dict[int, bool], reason: str = "GPUUnhealthy", why: str = "") -> None:
        """Apply several health changes at once: one ListAndWatch update, one node publish and one
        Event (``reason``) per newly unhealthy physical GPU (the time slices of a GPU flip together)."""
        changed: Dict[int, bool] = {}
        with self._cond:
            for index, healthy in states.items():
                if self._health.get(index) == healthy:
                    continue
                self._health[index] = healthy
                self.topology.gpus[index].healthy = healthy
                changed[index] = healthy
            if not changed:
                return
            self._version += 1
            self._cond.notify_all()
        reported = set()
        for index, healthy in sorted(changed.items()):
            log.warning("device %d is now %s", index, "Healthy" if healthy else "Unhealthy")
            self.metrics.health(index, healthy)
            g = self.topology.gpus[index]
            if self.api is not None and self.cfg.node_name and not healthy and g.physical not in reported:
                reported.add(g.physical)
                devs = sorted(i for i in changed if self.topology.gpus[i].physical == g.physical)
                record_event(self.api, {"kind": "Node", "metadata": {"name": self.cfg.node_name}}, reason,
                             f"device{'s' if len(devs) > 1 else ''} {format_group(devs)} ({g.bdf or 'no bdf'}) Unhealthy"
                             + (f": {why}" if why else ""),
                             "Warning", component="gpu-topology-device-plugin", host=self.cfg.node_name)
        self._publish_node()

    # ------------------------------------------------------------------ operator cordon
    CORDON_HOLD = "cordoned by the operator"

    def cordoned_from(self, value: str) -> Tuple[Set[int], List[str]]:
        """Devices ``<prefix>/cordoned-gpus`` names -> (indices, tokens that name no device here).  An
        index or a PCI address (``0000:75:00.0``, or without the domain) stands for its whole physical
        GPU: every partition or time slice of it."""
        t = self.topology
        by_bdf: Dict[str, int] = {}
        for g in t.gpus:
            if g.bdf:
                b = g.bdf.lower()
                by_bdf.setdefault(b, g.index)
                by_bdf.setdefault(b.split(":", 1)[1] if b.count(":") == 2 else b, g.index)
        out: Set[int] = set()
        unknown: List[str] = []
        for tok in (x.strip() for x in str(value or "").split(",")):
            if not tok:
                continue
            i: Optional[int] = None
            if tok.isascii() and tok.isdigit() and int(tok) < t.n:  # not str.isdigit alone: "¹" is a digit to it
                i = int(tok)
            elif ":" in tok:
                i = by_bdf.get(tok.lower())
            if i is None:
                unknown.append(tok)
                continue
            out |= {g.index for g in t.gpus if g.physical == t.gpus[i].physical}
        return out, unknown

    def apply_cordon(self, value: Optional[str]) -> Tuple[Set[int], Set[int]]:
        """Hold the devices the annotation names Unhealthy, release the ones it no longer names ->
        (newly cordoned, released).  A released device is Healthy again unless another hold (a GPU
        reset) or the next health pass says otherwise."""
        want, unknown = self.cordoned_from(value or "")
        with self._cond:
            add, drop = want - self._cordon_want, self._cordon_want - want
            self._cordon_want = set(want)
            for i in add:
                self._holds.setdefault(i, self.CORDON_HOLD)  # a reset hold stays; the reset's end turns it into this
            for i in drop:
                if self._holds.get(i) == self.CORDON_HOLD:  # a reset in progress keeps its own hold
                    self._holds.pop(i)
            released = {i for i in drop if i not in self._holds}
        node = {"kind": "Node", "metadata": {"name": self.cfg.node_name}}
        if unknown and unknown != self._cordon_unknown and self.api is not None and self.cfg.node_name:
            record_event(self.api, node, "GPUCordonUnknown", f"{self.cfg.contract.cordon_key} names no device here: "
                         f"{','.join(unknown)}", "Warning", component="gpu-topology-device-plugin", host=self.cfg.node_name)
        self._cordon_unknown = unknown
        if add:
            self.set_health_many({i: False for i in add}, reason="GPUCordoned", why=self.CORDON_HOLD)
        if released:
            states = {i: True for i in released}
            if self.health_fn is not None and states:
                try:
                    verdict = self.health_fn(self.topology)
                    states = {i: bool(verdict.get(i, True)) for i in states}
                except Exception as e:  # noqa: BLE001 - the next health pass decides
                    log.warning("health check after an uncordon failed: %s", e)
            self.set_health_many(states)
            if self.api is not None and self.cfg.node_name:
                record_event(self.api, node, "GPUUncordoned", f"devices {format_group(sorted(released))} back in service",
                             "Normal", component="gpu-topology-device-plugin", host=self.cfg.node_name)
        self.metrics.cordoned.set(len(want))
        return add, released

    def poll_node(self) -> Optional[dict]:
        """One GET of this plugin's own Node (the daemon's periodic label check): applies the operator's
        cordon and returns the object (None without an apiserver or on error)."""
        if self.api is None or not self.cfg.node_name:
            return None
        try:
            node = self.api.get_node(self.cfg.node_name)
        except Exception as e:  # noqa: BLE001 - the next poll retries
            log.warning("reading node %s failed: %s", self.cfg.node_name, e)
            return None
        self.apply_cordon(obj_annotations(node).get(self.cfg.contract.cordon_key))
        return node

    def update_topology(self, topo: Topology) -> None:
        """New probe results / partition change: re-publish and re-advertise."""
        with self._cond:
            self.topology = topo
            self._health = {g.index: bool(g.healthy) for g in topo.gpus}
            self._version += 1
            self._cond.notify_all()
        self.metrics.set_topology(topo)
        self.write_cdi_spec()
        self._publish_node()

    # ------------------------------------------------------------------ link re-measurement
    def node_idle(self) -> bool:
        """No live pod on this node holds (or is assumed to hold) a device — the only time a probe may
        run, since it saturates every xGMI link.  Unknown (no apiserver) counts as busy."""
        if self.api is None or not self.cfg.node_name:
            return False
        return node_is_idle(self.api, self.cfg.node_name, self._resource_names())

    def _resource_names(self) -> Tuple[str, ...]:
        """Every resource name a pod holding this node's devices may have asked for: the advertised
        one, its aliases, and both pools (whole GPUs and time slices) of the contract."""
        names = [self.cfg.resource_name] + list(self.cfg.resource_aliases)
        names += [self.cfg.contract.resource_name, self.cfg.contract.slice_resource]
        return tuple(dict.fromkeys(n for n in names if n))

    @staticmethod
    def link_change(old: Topology, new: Topology) -> float:
        """Largest relative change of a measured pair between two probes (inf if the measured set differs)."""
        if old.bw_gbps is None or new.bw_gbps is None or old.n != new.n:
            return float("inf")
        a, b = old.bw_gbps, new.bw_gbps
        fa, fb = np.isfinite(a), np.isfinite(b)
        np.fill_diagonal(fa, False)
        np.fill_diagonal(fb, False)
        if (fa != fb).any():
            return float("inf")
        if not fa.any():
            return 0.0
        return float(np.max(np.abs(b[fa] - a[fa]) / np.maximum(a[fa], 1e-9)))

    def _mark_probing(self, until: Optional[float]) -> bool:
        """Set (``until`` = deadline) or clear (None) the node's ``<prefix>/probing`` mark, which the
        extender's filter, sort and bind honour.  -> whether the apiserver took it."""
        if self.api is None or not self.cfg.node_name:
            return False
        try:
            self.api.patch_node(self.cfg.node_name, annotations={
                self.cfg.contract.probing_key: None if until is None else str(int(math.ceil(until)))})
            return True
        except Exception as e:  # noqa: BLE001 - an unmarked node is never probed; a stale mark expires
            log.warning("%s the probing mark on %s failed: %s", "clearing" if until is None else "setting",
                        self.cfg.node_name, e)
            return False

    @contextlib.contextmanager
    def allocation_hold(self):
        """Hold Allocate while a partition switch (deviceplugin/repartition.py) may run.  The yielded
        :class:`AllocationHold` tells the switch whether an Allocate is waiting (it then abandons the
        switch, and the Allocate proceeds on the unchanged layout); the switch sets ``started`` and
        ``switched``.  An Allocate held across a switch that changed the layout is refused: its device
        IDs name the old layout, and the plugin restarts to advertise the new one."""
        h = AllocationHold()
        with self._alloc_cond:
            self._hold = h
        try:
            yield h
        finally:
            with self._alloc_cond:
                self._hold = None
                if h.switched:
                    self._stale_layout = "the node's GPUs were repartitioned; the plugin restarts with new device IDs"
                self._alloc_cond.notify_all()

    def _call_reprobe(self):
        """``reprobe_fn(cancel=event)`` when it takes a cancel event (the child-process probe kills its
        child when an Allocate arrives), else ``reprobe_fn()``."""
        import inspect

        try:
            takes_cancel = "cancel" in inspect.signature(self.reprobe_fn).parameters
        except (TypeError, ValueError):
            takes_cancel = False
        return self.reprobe_fn(cancel=self._cancel) if takes_cancel else self.reprobe_fn()

    def reprobe(self) -> bool:
        """One idle-time re-measurement; republish if the links moved.  -> republished.

        The kubelet never retries a failed ``Allocate`` (the pod is rejected for good), so a probe must
        not refuse one.  Instead (``design.md:236-246``: Allocate hands a pod its devices):
          1. the node is marked ``<prefix>/probing: <deadline>``, so the extender stops choosing it;
          2. after ``probe_settle_s`` (a bind already past the extender's check lands in that window)
             the node must still be idle, or the mark is cleared and nothing runs;
          3. an ``Allocate`` arriving while the probe runs cancels it (the probe child is killed) and
             waits, at most ``probe_yield_s``, for the links to be released, then proceeds;
          4. the mark is cleared; a cancelled probe, or one a pod arrived during, is discarded (its
             traffic would skew the matrix)."""
        if self.reprobe_fn is None:
            return False
        if not self.maintenance.acquire(blocking=False):  # a partition switch holds the GPUs
            self.metrics.reprobes.labels("busy").inc()
            return False
        try:
            return self._reprobe_locked()
        finally:
            self.maintenance.release()

    def _reprobe_locked(self) -> bool:
        if not self.node_idle():
            self.metrics.reprobes.labels("busy").inc()
            return False
        if not self._mark_probing(self.clock() + self.cfg.probe_mark_s):
            self.metrics.reprobes.labels("unmarked").inc()
            return False
        try:
            if self.cfg.probe_settle_s > 0 and self._stop.wait(self.cfg.probe_settle_s):
                return False
            with self._alloc_cond:
                if not self.node_idle():
                    self.metrics.reprobes.labels("busy").inc()
                    return False
                self._cancel = threading.Event()
                self._probing = True
            try:
                new = self._call_reprobe()
            finally:
                with self._alloc_cond:
                    self._probing = False
                    cancelled = self._cancel.is_set()
                    still_idle = self.node_idle()
                    self._alloc_cond.notify_all()
        finally:
            self._mark_probing(None)
        self.reprobes += 1
        if cancelled:
            log.warning("link re-probe: cancelled by an Allocate; the measurement is discarded")
            self.metrics.reprobes.labels("cancelled").inc()
            return False
        if not still_idle:
            log.warning("link re-probe: a pod claimed devices during the probe; discarding the measurement")
            self.metrics.reprobes.labels("discarded").inc()
            return False
        if new is None or new.n != self.topology.n:
            log.warning("link re-probe produced no usable topology")
            self.metrics.reprobes.labels("failed").inc()
            return False
        # noise-equivalent links take their class value, kept from the published matrix while the new
        # median stays within the band (ops/checks.py band_links): a healthy node republishes nothing
        from ..ops.checks import apply_banding

        apply_banding(new, prev=self.topology)
        delta = self.link_change(self.topology, new)
        if delta <= self.cfg.reprobe_tolerance:
            log.info("link re-probe: largest change %.1f%% (within tolerance)", 100 * delta)
            self.metrics.reprobes.labels("unchanged").inc()
            return False
        for g in new.gpus:  # health is the RAS monitor's call, not the probe's
            g.healthy = self._health.get(g.index, True)
        new.node_name = self.topology.node_name
        log.warning("link re-probe: largest change %s; republishing the measured matrix",
                    "in the measured set" if delta == float("inf") else f"{100 * delta:.1f}%")
        self.update_topology(new)
        self.republished += 1
        self.metrics.reprobes.labels("republished").inc()
        return True

    # ------------------------------------------------------------------ node publication (A5, B7)
    def _publish_node(self) -> None:
        if not (self.api is not None and self.cfg.publish_node and self.cfg.node_name):
            return
        t = self.topology
        c = self.cfg.contract
        models = sorted({g.model for g in t.gpus})
        labels = {
            c.label_model: models[0] if len(models) == 1 else "mixed",
            c.label_partition: t.gpus[0].partition if t.gpus else "",
            c.label_gfx: t.gpus[0].gfx if t.gpus else "",
            c.label_slices: str(max((int((t.physical == p).sum()) for p in set(t.physical.tolist())), default=1)),
            **tm_labels(self.cfg.topology_manager, c.prefix),
        }
        ann = encode_node_annotations(t, c)
        ann[c.active_slices_key] = str(slices_per_gpu(t))  # the layout a restart must keep while pods hold devices
        self.metrics.annotation_bytes.set(sum(len(k) + len(v) for k, v in ann.items()))
        try:
            self.api.patch_node(self.cfg.node_name, annotations=ann, labels=labels)
            self.metrics.node_publishes.labels("ok").inc()
        except Exception as e:
            self.metrics.node_publishes.labels("error").inc()
            log.warning("publishing topology on node %s failed: %s", self.cfg.node_name, e)

    # ------------------------------------------------------------------ gRPC handlers
    def GetDevicePluginOptions(self, request, context):
        return pb.DevicePluginOptions(pre_start_required=self.cfg.prestart_validate, get_preferred_allocation_available=True)

    def ListAndWatch(self, request, context):
        last = -1
        while not self._stop.is_set() and context.is_active():
            with self._cond:
                if self._version == last:
                    self._cond.wait(timeout=0.5)
                    if self._version == last:
                        continue
                last = self._version
                devs = self.devices()
            yield pb.ListAndWatchResponse(devices=devs)

    def GetPreferredAllocation(self, request, context):
        """The kubelet asks once per container, with that container's count.  The answer
        is the part of the extender's GROUP this container should get: the pod whose next container
        asks for ``size`` devices (in-progress admissions first, then the oldest ASSUME_TIME), its
        devices the kubelet still offers, and — when the container gets only part of the GROUP — the
        best sub-placement of them that contains the devices an init container handed on
        (``must_include``)."""
        resp = pb.PreferredAllocationResponse()
        with self._alloc_lock:  # the admission records are Allocate's
            cands, live = self._admission_view()
        for creq in request.container_requests:
            avail = self._ids(context, creq.available_deviceIDs)
            must = self._ids(context, creq.must_include_deviceIDs)
            size = int(creq.allocation_size)
            with self._alloc_lock:
                self._gpa_must = (self._gpa_must or set()) | set(must)
            ids = self._preferred_from_group(cands, live, size, avail, must)
            if ids is not None:
                self.metrics.preferred.labels("annotation").inc()
            else:
                ids = self._preferred_fallback(size, avail, must)
            resp.container_responses.add(deviceIDs=[str(i) for i in ids])
        return resp

    def _preferred_from_group(self, cands: List["_Candidate"], live: Dict[str, dict], size: int, avail: Sequence[int],
                              must: Sequence[int]) -> Optional[List[int]]:
        avail_s, must_s = set(avail), set(must)
        rec = self._reuse(must) if must_s else None
        if rec is not None and rec.key in live:  # reused devices: the pod of the previous call
            pa = PodAssignment.from_annotations(obj_annotations(live[rec.key]))
            pick = self._pick_part(set(pa.group) | rec.claimed, size, avail_s, must_s) if pa is not None else None
            if pick is not None:
                return pick
        for c in cands:
            if c.pa is None:
                continue
            nxt = c.next_size()
            if nxt is None and len(set(c.pa.group) & avail_s) != size:
                continue  # no per-container request known: only a GROUP of exactly this size
            if nxt is not None and nxt != size:
                continue
            pick = self._pick_part(set(c.pa.group), size, avail_s, must_s)
            if pick is not None:
                return pick
        return None

    def _pick_part(self, g: set, size: int, avail_s: set, must_s: set) -> Optional[List[int]]:
        """``size`` devices of GROUP ``g`` the kubelet offers, ``must_s`` among them: all of them, or
        the best sub-placement when the container gets only part of the GROUP.  None if they do not fit."""
        free = g & avail_s
        if not must_s <= g or len(free) < size:
            return None
        if len(free) == size:
            return sorted(free)
        healthy = sorted(i for i in free if self._health.get(i, True))
        try:
            return sorted(select_with(self.topology, size, healthy, sorted(must_s), self.cfg.policy))
        except (NoFeasiblePlacement, ValueError, AssertionError):
            rest = [i for i in sorted(free, key=lambda i: (i not in healthy, i)) if i not in must_s]
            return sorted(list(must_s) + rest[: size - len(must_s)])

    def _preferred_fallback(self, size: int, avail: Sequence[int], must: Sequence[int]) -> List[int]:
        """No annotated pod matches: run the placement core over the healthy available devices.  A
        placement error never fails admission (the kubelet would reject the pod): the answer then
        degrades to must-include first, then the lowest available ids."""
        healthy = [a for a in avail if 0 <= a < self.topology.n and self._health.get(a, True)]
        try:
            ids = list(select_with(self.topology, size, healthy, must, self.cfg.policy))
            self.metrics.preferred.labels("placement").inc()
            return ids
        except (NoFeasiblePlacement, ValueError, AssertionError) as e:
            log.warning("GetPreferredAllocation: placement failed (%s); answering in id order", e)
            self.metrics.preferred.labels("fallback").inc()
            out = [m for m in must if m in avail][:size]
            out += [a for a in sorted(avail, key=lambda a: (a not in healthy, a)) if a not in out][: size - len(out)]
            return sorted(out)

    def _ids(self, context, raw) -> List[int]:
        """Device IDs of a kubelet request: the decimal indices ListAndWatch advertised; anything else
        is refused as INVALID_ARGUMENT (not an UNKNOWN error out of int())."""
        try:
            return [int(x) for x in raw]
        except (TypeError, ValueError):
            self._refuse(context, grpc.StatusCode.INVALID_ARGUMENT, f"device ids {list(raw)} are not this plugin's", "invalid")
            raise  # context.abort raised already; a stub context that does not must not go on either

    def _refuse(self, context, code, msg: str, outcome: str) -> None:
        self.metrics.allocations.labels(outcome).inc()
        if self.api is not None and self.cfg.node_name:
            record_event(self.api, {"kind": "Node", "metadata": {"name": self.cfg.node_name}}, "FailedGPUAllocate", msg,
                         "Warning", component="gpu-topology-device-plugin", host=self.cfg.node_name)
        context.abort(code, msg)

    def Allocate(self, request, context):
        t0 = time.perf_counter()
        resp = pb.AllocateResponse()
        all_ids: List[int] = []
        for creq in request.container_requests:
            ids = self._ids(context, creq.devices_ids)
            bad = [i for i in ids if i < 0 or i >= self.topology.n]
            if bad:
                self._refuse(context, grpc.StatusCode.INVALID_ARGUMENT, f"unknown device ids {bad}", "invalid")
            unhealthy = [i for i in ids if not self._health.get(i, True)]
            if unhealthy:
                self._refuse(context, grpc.StatusCode.FAILED_PRECONDITION, f"devices {unhealthy} are unhealthy", "unhealthy")
            all_ids.extend(ids)
        missing = self._missing_device_nodes(all_ids)
        if missing:
            self._refuse(context, grpc.StatusCode.FAILED_PRECONDITION, f"device nodes missing on this node: {missing}", "missing")
        with self._alloc_cond:
            if self._hold is not None:
                h = self._hold
                h.waiters += 1
                self.metrics.allocations.labels("switch_wait").inc()
                try:
                    while self._hold is h:
                        self._alloc_cond.wait(1.0)
                finally:
                    h.waiters -= 1
            if self._stale_layout:
                self._alloc_cond.release()  # _refuse aborts the RPC (raises); never hold the lock across it
                try:
                    self._refuse(context, grpc.StatusCode.UNAVAILABLE, self._stale_layout, "stale_layout")
                finally:
                    self._alloc_cond.acquire()
            if self._probing:
                # never refuse (the kubelet would reject the pod for good): the probe yields — its
                # child is killed — and the container starts once the links are released
                self._cancel.set()
                self.metrics.allocations.labels("probe_yield").inc()
                deadline = time.monotonic() + self.cfg.probe_yield_s
                while self._probing and time.monotonic() < deadline:
                    self._alloc_cond.wait(deadline - time.monotonic())
                if self._probing:
                    log.warning("Allocate of %s: the link probe did not yield within %.0fs; allocating anyway",
                                sorted(set(all_ids)), self.cfg.probe_yield_s)
            # the kubelet sends one container per call; each container request is one step of its pod
            pods = []
            for creq in request.container_requests:
                ids = sorted({int(x) for x in creq.devices_ids})
                reused = set(ids) if self._gpa_must is None else self._gpa_must & set(ids)
                if self._gpa_must is None and self.cfg.topology_manager.active and not self._continuing():
                    # a Topology Manager skips GetPreferredAllocation also for a new pod whose aligned
                    # devices are exactly its need: with no admission under way this is no reuse, even
                    # when the GPUs are those a pod that just ended (status not updated yet) freed
                    reused = set()
                self._claimed_by = None
                pods.append(self._claim_pod(ids, reused))
                self._link(ids, self._claimed_by, reused)
            self._gpa_must = None
            self._last_alloc = time.monotonic()
        for creq, pod in zip(request.container_requests, pods):
            ids = [int(x) for x in creq.devices_ids]
            resp.container_responses.append(self._container_response(ids, self._rccl_env(pod) if pod is not None else {}))
        pod = next((p for p in pods if p is not None), None)
        self.allocations.append((f"{meta(pod).get('namespace')}/{meta(pod).get('name')}" if pod else "", tuple(sorted(all_ids))))
        self.metrics.allocations.labels("ok").inc()
        self.metrics.allocated_devices.inc(len(all_ids))
        self.metrics.allocate_seconds.observe(time.perf_counter() - t0)
        return resp

    def PreStartContainer(self, request, context):
        """Placement validation (flow step 8): an exact-checked RCCL all-reduce over the container's
        devices, in a child process (the plugin never holds HIP contexts).  A failure fails the
        container start (the kubelet retries it) and is recorded as an Event; a success writes the
        measured bandwidth on the pod.  A no-op unless ``prestart_validate``."""
        if not self.cfg.prestart_validate:
            return pb.PreStartContainerResponse()
        ids = sorted(set(self._ids(context, request.devices_ids)))
        t0 = time.perf_counter()
        try:
            res = self.validate_fn(ids)
        except Exception as e:  # noqa: BLE001 - reported to the kubelet below
            res = {"ok": False, "error": str(e)}
        self.metrics.validate_seconds.observe(time.perf_counter() - t0)
        ok = bool(res.get("ok")) and int(res.get("wrong", 0)) == 0
        self.metrics.validations.labels("ok" if ok else "failed").inc()
        pod = self._assigned_pod(ids)
        if not ok:
            msg = f"RCCL validation of devices {ids} failed: {res.get('error') or str(res.get('wrong')) + ' wrong elements'}"
            record_event(self.api, pod if pod is not None else {"kind": "Node", "metadata": {"name": self.cfg.node_name}},
                         "FailedGPUPlacementValidation", msg, "Warning", component="gpu-topology-device-plugin",
                         host=self.cfg.node_name)
            context.abort(grpc.StatusCode.FAILED_PRECONDITION, msg)
        if pod is not None and self.api is not None and self._widest_validation(pod, res):
            md = meta(pod)
            rec = {k: res[k] for k in ("k", "peak_bytes", "peak_algbw_gbps", "peak_busbw_gbps") if k in res}
            rec["devices"] = format_group(ids)
            ann = {self.cfg.contract.validated_key: json.dumps(rec, separators=(",", ":"))}
            try:
                self.api.patch_pod_annotations(md.get("namespace", "default"), md["name"], ann)
            except Exception as e:  # noqa: BLE001 - the validation passed; the record is best effort
                log.warning("recording validation on %s failed: %s", md.get("name"), e)
        return pb.PreStartContainerResponse()

    def _widest_validation(self, pod: dict, res: Dict[str, object]) -> bool:
        """Whether ``res`` should be the pod's validation record: each container start (a restart too)
        validates that container's devices, and the pod keeps its widest one (ties: the latest), so a
        one-GPU sidecar does not overwrite the all-reduce of a four-GPU container."""
        old = obj_annotations(pod).get(self.cfg.contract.validated_key)
        if not old:
            return True
        try:
            return int(res.get("k", 0)) >= int(json.loads(old).get("k", 0))
        except (ValueError, TypeError, AttributeError):
            return True

    def _assigned_pod(self, ids: Sequence[int]) -> Optional[dict]:
        """The live pod on this node whose confirmed GROUP holds ``ids`` (one container's devices;
        newest ASSUME_TIME)."""
        best = None
        for p in self._node_pods():
            pa = PodAssignment.from_annotations(obj_annotations(p))
            if pa is not None and pa.assigned and set(ids) <= set(pa.group):
                if best is None or pa.assume_time >= best[1]:
                    best = (p, pa.assume_time)
        return best[0] if best else None

    def _validate_in_child(self, ids: Sequence[int]) -> Dict[str, object]:
        """``gtk validate`` over ``ids`` (node indices, resolved to HIP ordinals by PCI address) in a
        child process: 1 MiB..64 MiB bf16 all-reduces, exact-checked; returns its summary line."""
        import subprocess
        import sys

        ids = physical_group(self.topology, ids)  # time slices of one GPU validate that GPU once
        bdfs = ",".join(self.topology.gpus[self._first_slice(i)].bdf for i in ids)
        cmd = [sys.executable, "-m", "gpu_topology_on_k8s_amd", "validate", "--group", ",".join(map(str, ids)),
               "--min-bytes", str(1 << 20), "--max-bytes", str(64 << 20), "--factor", "8", "--iters", "5", "--warmup", "2"]
        if all(self.topology.gpus[self._first_slice(i)].bdf for i in ids):
            cmd += ["--bdfs", bdfs]
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        try:
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=self.cfg.validate_timeout, cwd=root)
        except subprocess.TimeoutExpired:
            return {"ok": False, "error": f"validation timed out after {self.cfg.validate_timeout:.0f}s"}
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{"summary"')]
        if not lines:
            return {"ok": False, "error": f"validate exited {p.returncode}: {(p.stderr or p.stdout).strip()[-300:]}"}
        out = json.loads(lines[-1])
        out["ok"] = p.returncode == 0
        return out

    # ------------------------------------------------------------------ Allocate helpers
    def _first_slice(self, physical: int) -> int:
        """Topology index of the first device of physical GPU ``physical`` (itself on an SPX node)."""
        return next(g.index for g in self.topology.gpus if g.physical == physical)

    def device_nodes(self, ids: Sequence[int]) -> List[Tuple[str, str]]:
        """(container path, host path) of every device node the container needs for ``ids``, each
        once (time slices of one GPU share its render/card nodes)."""
        root = self.cfg.dev_root.rstrip("/")
        out = [("/dev/kfd", f"{root}/kfd")]
        for i in ids:
            g = self.topology.gpus[i]
            minor = g.render_node
            out.append((f"/dev/dri/renderD{minor}", f"{root}/dri/renderD{minor}"))
            if g.card >= 0:
                out.append((f"/dev/dri/card{g.card}", f"{root}/dri/card{g.card}"))
        return list(dict.fromkeys(out))

    @staticmethod
    def _optional_node(container_path: str) -> bool:
        """ROCm compute needs ``/dev/kfd`` and the render nodes; a ``card<N>`` (primary / display) node
        is handed over when the node has it, and its absence never refuses a pod.  Found on MI355X:
        a container given only ``renderD128`` had no ``card16`` although amdsmi names it
        (``bench/plugin_soak.py``), and strict mode refused every Allocate there."""
        return container_path.startswith("/dev/dri/card")

    def _missing_device_nodes(self, ids: Sequence[int]) -> List[str]:
        if self.cfg.device_specs != "strict":
            return []
        return [h for c, h in self.device_nodes(ids) if not self._optional_node(c) and not os.path.exists(h)]

    def _container_response(self, ids: Sequence[int], extra_env: Dict[str, str]) -> pb.ContainerAllocateResponse:
        r = pb.ContainerAllocateResponse()
        if self.cfg.device_specs == "cdi":
            from .cdi import cdi_name

            # one name per physical device: time slices of a GPU share its nodes (topology/shares.py)
            for i in dict.fromkeys(self._first_slice(self.topology.gpus[i].physical) if self.topology.gpus[i].shares > 1 else i
                                   for i in ids):
                r.cdi_devices.add(name=cdi_name(self.cfg.cdi_kind, i))
        for cpath, hpath in ([] if self.cfg.device_specs == "cdi" else self.device_nodes(ids)):
            if (self.cfg.device_specs == "stub" or self._optional_node(cpath)) and not os.path.exists(hpath):
                continue  # kind / fake GPUs, or an absent card node: never hand containerd a missing host path
            r.devices.add(container_path=cpath, host_path=hpath, permissions="rw")
        numa = {int(self.topology.gpus[i].numa) for i in ids}
        mask = ""
        if slices_per_gpu(self.topology) > 1:
            # time slices (topology/shares.py): the container sees the physical GPUs behind them, and
            # its share of each (GTK_GPU_FRACTION, in GROUP order) caps its HBM cooperatively
            frac = share_fractions(self.topology, ids)
            group = sorted(frac)
            r.envs[ENV_GROUP] = format_group(group)
            r.envs[ENV_BDFS] = ",".join(self.topology.gpus[self._first_slice(p)].bdf for p in group)
            r.envs[ENV_FRACTION] = ",".join(f"{frac[p]:.4g}" for p in group)
            r.envs[ENV_SLICES] = format_group(ids)
            mask = cu_mask_env(self.topology, ids) if self.cfg.share_cu_mask else ""
        else:
            r.envs[ENV_GROUP] = format_group(ids)
            # PCI addresses in GROUP order: HIP renumbers the container's devices 0..k-1, so tools inside
            # the pod map GROUP -> HIP ordinal by address (topology/identity.py, `gtk validate`)
            r.envs[ENV_BDFS] = ",".join(self.topology.gpus[i].bdf for i in ids)
        r.envs["GTK_NUMA_NODES"] = ",".join(str(x) for x in sorted(numa))
        cpuset = recommended_cpuset(self.topology, ids)  # Gaia B6: the devices' local core slices
        if cpuset:
            r.envs["GTK_CPUSET"] = cpuset
        nics = self.topology.nearest_nics(ids) if self.cfg.nic_env else []
        if nics:
            r.envs["GTK_NICS"] = ",".join(nics)
            r.envs["NCCL_IB_HCA"] = "=" + ",".join(nics)  # exact-name match
        if self.cfg.container_ipc_mode:  # before the pod's own env (rccl-env), which may override it
            r.envs["HSA_ENABLE_IPC_MODE_LEGACY"] = self.cfg.container_ipc_mode
        for k, v in extra_env.items():
            r.envs[k] = v
        if mask:  # after the pod's own RCCL/HSA env: its queues run on its slices' CUs, disjoint from its neighbours'
            r.envs["HSA_CU_MASK"] = mask
        if slices_per_gpu(self.topology) > 1 and self._guard_ready:
            self._guard_container(r, ids, mask)
        r.annotations["gputopology.amd.com/devices"] = format_group(ids)
        return r

    # ------------------------------------------------------------------ share guard (vGPU container tier)
    GUARD_LIB_IN_CONTAINER = "/usr/local/lib/gtk-vgpu/libgtk_vgpu.so"
    GUARD_CONF_IN_CONTAINER = "/etc/gtk-vgpu.conf"
    GUARD_ACCT_IN_CONTAINER = "/var/run/gtk-vgpu.acct"  # pod-wide budget: one accounting table per allocation

    def install_guard(self) -> bool:
        """Copy the guard library into ``guard_dir`` (atomically: a running pod keeps the file it
        mapped).  -> ready.  A missing library leaves shares cooperative and says so."""
        self._guard_ready = False
        if self.cfg.share_guard == "off" or slices_per_gpu(self.topology) <= 1:
            return False
        import shutil

        src = self.cfg.guard_lib
        if src is None:
            from .._native import NativeUnavailable, binary

            try:
                src = str(binary("libgtk_vgpu.so"))
            except NativeUnavailable as e:
                log.warning("share guard requested but unavailable (%s): time-sliced shares stay cooperative", e)
                return False
        try:
            os.makedirs(os.path.join(self.cfg.guard_dir, "alloc"), exist_ok=True)
            dst = os.path.join(self.cfg.guard_dir, "libgtk_vgpu.so")
            tmp = f"{dst}.tmp{os.getpid()}"
            shutil.copyfile(src, tmp)
            os.chmod(tmp, 0o755)
            os.replace(tmp, dst)
            with open(os.path.join(self.cfg.guard_dir, "ld.so.preload"), "w") as f:
                f.write(self.GUARD_LIB_IN_CONTAINER + "\n")
        except OSError as e:
            log.warning("installing the share guard into %s failed (%s): shares stay cooperative", self.cfg.guard_dir, e)
            return False
        self._guard_ready = True
        return True

    def guard_config(self, ids: Sequence[int], mask: str, acct: bool = True) -> str:
        """The guard's config for a container holding the time slices ``ids``: per partly held GPU the
        HBM of the slices it holds and their CUs, and the accounting file every process of the pod
        shares (one budget for the pod, not per process).  GPUs are named by PCI address (an
        ordinal moves when the pod sets ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES); only when discovery
        found no address does the config fall back to the container ordinal (position among the held
        physical GPUs) and the HSA_CU_MASK value Allocate computed."""
        frac = share_fractions(self.topology, ids)
        cus = share_cus(self.topology, ids) if mask else {}
        lines = ["# gtk-vgpu: written by the device plugin at Allocate (deviceplugin/plugin.py)"]
        partial = [p for p in sorted(frac) if frac[p] < 1.0]
        held = {p: [self.topology.gpus[int(i)] for i in ids if self.topology.gpus[int(i)].physical == p] for p in partial}
        by_address = all(held[p] and held[p][0].bdf for p in partial)
        for ordinal, p in enumerate(sorted(frac)):
            if p not in held:
                continue
            hbm = sum(int(g.vram_bytes) for g in held[p])
            if by_address:
                # the container ordinal follows as the guard's fallback, used only when the runtime
                # enumerates no GPU with that address (vgpu_guard.cpp: reported, never silently dropped)
                bdf = held[p][0].bdf
                if hbm > 0:
                    lines.append(f"hbm_limit_bdf {bdf} {hbm} {ordinal}")
                if p in cus:
                    lines.append(f"cu_mask_bdf {bdf} {format_cus(cus[p])} {ordinal}")
            elif hbm > 0:
                lines.append(f"hbm_limit {ordinal} {hbm}")
        if mask and not by_address:
            lines.append(f"cu_mask {mask}")
        if acct:
            lines.append(f"acct {self.GUARD_ACCT_IN_CONTAINER}")
        return "\n".join(lines) + "\n"

    def _guard_container(self, r: pb.ContainerAllocateResponse, ids: Sequence[int], mask: str) -> None:
        frac = share_fractions(self.topology, ids)
        if all(f >= 1.0 for f in frac.values()):
            return  # whole GPUs only: nothing to guard
        conf, acct = self._guard_files(ids, mask)
        r.mounts.add(container_path=self.GUARD_LIB_IN_CONTAINER, host_path=os.path.join(self.cfg.guard_dir, "libgtk_vgpu.so"),
                     read_only=True)
        r.mounts.add(container_path=self.GUARD_CONF_IN_CONTAINER, host_path=conf, read_only=True)
        r.mounts.add(container_path=self.GUARD_ACCT_IN_CONTAINER, host_path=acct, read_only=False)
        r.envs["GTK_VGPU_CONFIG"] = self.GUARD_CONF_IN_CONTAINER
        if self.cfg.share_guard == "preload":  # loaded by every process whatever its env says
            r.mounts.add(container_path="/etc/ld.so.preload", host_path=os.path.join(self.cfg.guard_dir, "ld.so.preload"),
                         read_only=True)
        # and LD_PRELOAD in both modes: the dynamic loader maps the library once either way
        r.envs["LD_PRELOAD"] = self.GUARD_LIB_IN_CONTAINER
        self.metrics.guarded.inc()

    def _guard_files(self, ids: Sequence[int], mask: str) -> Tuple[str, str]:
        """A config and an accounting table of their own for this allocation.  The names are unique:
        a process of an earlier holder of these slices (a terminating pod, a sidecar that keeps its
        devices) may still map its own table, and truncating a mapped file would SIGBUS it and wipe the
        pod's budget.  Older files of the same slices are removed once no process holds a
        slot lock in their table (every live guarded process holds one): by then the kubelet has handed
        the slices to this allocation, so the pod that owned them is gone."""
        d = os.path.join(self.cfg.guard_dir, "alloc")
        os.makedirs(d, exist_ok=True)
        key = "slices-" + "-".join(str(int(i)) for i in sorted(set(ids)))
        seq = next(self._guard_seq)  # itertools.count: atomic under the GIL
        base = os.path.join(d, f"{key}.{time.time_ns():x}.{os.getpid():x}.{seq}")
        conf, acct = base + ".conf", base + ".acct"
        tmp = f"{conf}.tmp"
        with open(tmp, "w") as f:
            f.write(self.guard_config(ids, mask))
        os.replace(tmp, conf)
        fd = os.open(acct, os.O_RDWR | os.O_CREAT | os.O_EXCL, 0o666)  # world-writable: any container user
        os.fchmod(fd, 0o666)
        os.close(fd)
        self._gc_guard_files(d, set(int(i) for i in ids), keep=base)
        return conf, acct

    @staticmethod
    def _acct_in_use(path: str) -> bool:
        """Some process holds a record lock in the table (a live guarded process owns a slot)."""
        import fcntl

        try:
            fd = os.open(path, os.O_RDWR)
        except OSError:
            return False
        try:
            fcntl.lockf(fd, fcntl.LOCK_EX | fcntl.LOCK_NB, 0, 0)  # the whole file, no wait
        except OSError:
            return True
        finally:
            os.close(fd)  # closing drops the probe lock
        return False

    def _gc_guard_files(self, d: str, ids: set, keep: str) -> None:
        for name in os.listdir(d):
            if not name.endswith(".acct") or not name.startswith("slices-"):
                continue
            base = os.path.join(d, name[:-5])
            if base == keep:
                continue
            try:
                old = {int(x) for x in name.split(".", 1)[0][len("slices-"):].split("-")}
            except ValueError:
                continue
            if not old & ids or self._acct_in_use(base + ".acct"):
                continue
            for ext in (".acct", ".conf"):
                try:
                    os.unlink(base + ext)
                except FileNotFoundError:
                    pass

    def _rccl_env(self, pod: dict) -> Dict[str, str]:
        if not self.cfg.pass_rccl_env:
            return {}
        raw = obj_annotations(pod).get(f"{self.cfg.contract.prefix}/{RCCL_ENV_ANNOTATION_SUFFIX}", "")
        env = {}
        for line in raw.replace(";", "\n").splitlines():
            if "=" not in line:
                continue
            k, v = line.split("=", 1)
            k = k.strip()
            if k.startswith(_ENV_PREFIXES):
                env[k] = v.strip()
        return env

    def _node_pods(self, cached: bool = False) -> List[dict]:
        """This node's live pods.  ``cached``: from the apiserver's watch cache, for the periodic
        reconcile (on every node every --reconcile-interval: a consistent read would be an etcd range
        over every pod of the cluster each time; a stale answer only delays a correction, which is a
        conditional patch)."""
        if self.api is None or not self.cfg.node_name:
            return []
        try:
            return [p for p in self.api.list_pods(node_name=self.cfg.node_name, cached=cached) if not pod_is_terminal(p)]
        except Exception as e:
            log.warning("listing pods on %s failed: %s", self.cfg.node_name, e)
            return []

    def _admission_view(self) -> Tuple[List["_Candidate"], Dict[str, dict]]:
        """(candidates, live pods by key).  Candidates are the pending pods on this node the kubelet
        may be allocating for, in the order a container's request is matched against them: a pod whose
        admission is under way (some containers got devices; the kubelet admits one pod at a time),
        then the oldest ASSUME_TIME (the design's implicit rule), then pods scheduled around the
        extender (no GROUP) by creation time.  Pods whose GROUP is confirmed and whose containers have
        all been allocated are not candidates.  Live pods are the node's pods that may hold devices
        (not terminal, not being deleted).  Records of pods that are gone are dropped here."""
        names = self._resource_names()
        out: List[_Candidate] = []
        live: Dict[str, dict] = {}
        for p in self._node_pods():
            md = meta(p)
            key = f"{md.get('namespace', 'default')}/{md.get('name')}"
            if not md.get("deletionTimestamp"):
                live[key] = p
            pa = PodAssignment.from_annotations(obj_annotations(p))
            if pod_phase(p) != "Pending" and (pa is None or pa.assigned):
                # started: its containers have their devices.  A started pod whose GROUP was never
                # claimed stays a candidate: the kubelet admitted it with another pod's devices (out of
                # order), so its GROUP is what the other pod's containers will be given
                continue
            adm = self._admissions.get(key)
            if adm is not None and adm.uid != md.get("uid", ""):
                adm = None  # a new pod of the same name
            try:
                steps = pod_device_steps(p, names)
            except ValueError:
                steps = []
            if pa is None and not steps:
                continue
            if adm is None and pa is not None and pa.assigned:
                continue  # admitted before (or by a previous run of this plugin)
            out.append(_Candidate(p, key, pa, steps, adm))
        pending = {c.key for c in out}
        for key in [k for k in self._admissions if k not in pending]:
            del self._admissions[key]
        if self._chain is not None:
            # the kubelet frees a pod's devices only when the pod ends: while the pod the previous call
            # was matched to lives, a later call holding its devices is a reuse.  Once that pod ended (or
            # calls stopped coming) they may have been freed and handed to another pod, which is no reuse
            rec = self._chain[1]
            pod = live.get(rec.key) if rec is not None else None
            over = (time.monotonic() - self._last_alloc > self.cfg.admission_settle_s
                    or (rec is not None and (pod is None or meta(pod).get("uid", "") != rec.uid)))
            if over:
                self._chain = None
        out.sort(key=lambda c: (c.adm is None or c.adm.done == 0, c.pa is None,
                                float(c.pa.assume_time) if c.pa is not None else 0.0,
                                meta(c.pod).get("creationTimestamp", ""), meta(c.pod).get("name", "")))
        return out, live

    def _continuing(self) -> bool:
        """The previous Allocate's admission still has containers to allocate."""
        rec = self._chain[1] if self._chain is not None else None
        return rec is not None and self._admissions.get(rec.key) is rec

    def _reuse(self, reused: Sequence[int]) -> Optional[_Admission]:
        """The record of the previous Allocate when the devices the kubelet reused (``reused``: what
        GetPreferredAllocation was told to include, see ``_gpa_must``) are some of its unit's.  The
        kubelet admits one pod at a time and hands a regular init container's devices only to the
        later containers of the same pod, so such a call continues the previous call's admission —
        whichever pod that call was matched to."""
        if self._chain is None or not self._chain[0] & {int(d) for d in reused}:
            return None
        return self._chain[1]

    def _link(self, ids: Sequence[int], adm: Optional[_Admission], reused: Sequence[int] = ()) -> None:
        """Record one Allocate call in the admission units (see ``_unit_of``)."""
        ids_s = {int(d) for d in ids}
        linked = self._chain is not None and self._chain[0] & {int(d) for d in reused}
        unit = self._chain[0] | ids_s if linked else set(ids_s)
        for d in unit:
            self._unit_of[d] = unit
        self._chain = (unit, adm)

    def _match(self, cands: List["_Candidate"], ids: List[int]) -> Tuple[Optional["_Candidate"], str]:
        """The candidate one container's devices are for, and how it matched: ``group`` (inside its
        GROUP), ``resized`` (its next container asks this many, the kubelet chose other devices) or
        ``unannotated`` (scheduled around the extender)."""
        ids_s, n = set(ids), len(ids)
        for c in cands:  # devices of its GROUP, for a container of this size
            nxt = c.next_size()
            if c.pa is not None and ids_s <= set(c.pa.group) and (nxt == n or (nxt is None and c.adm is None)):
                return c, "group"
        for c in cands:  # the kubelet chose outside every GROUP: the pod whose next container asks n
            nxt = c.next_size()
            if c.pa is not None and (nxt == n or (nxt is None and len(set(c.pa.group)) == n and c.adm is None)):
                return c, "resized"
        for c in cands:
            if c.pa is None and c.next_size() == n:
                return c, "unannotated"
        return None, ""

    def _claim_pod(self, ids: List[int], reused: Sequence[int] = ()) -> Optional[dict]:
        """One container's ``Allocate``: find the pod the devices are for, record them against its
        GROUP, and flip it to ASSIGNED=true (conditional patch) once every device of the GROUP has been
        allocated — with one ``Allocate`` per container (the real kubelet), a pod is claimed over
        several calls.  A container reusing devices of an earlier container belongs to the same pod
        (:meth:`_reuse`).  When the kubelet chose devices outside the GROUP, the GROUP is rewritten to
        what it chose (the extender's view must be the kubelet's truth).  -> the pod (for its env)."""
        if self.api is None or not self.cfg.node_name:
            return None
        for attempt in range(5):
            cands, live = self._admission_view()
            rec = self._reuse(reused)
            if rec is not None and rec.key in live and meta(live[rec.key]).get("uid", "") == rec.uid:
                pod = live[rec.key]
                c = next((x for x in cands if x.key == rec.key), None)
                pa = PodAssignment.from_annotations(obj_annotations(pod))
                steps = c.steps if c is not None else []
                adm, how = rec, "reuse"
            else:
                c, how = self._match(cands, ids)
                if c is None:
                    log.warning("no pending pod on %s matches allocation %s", self.cfg.node_name, ids)
                    return None
                pod, pa, steps = c.pod, c.pa, c.steps
                adm = c.adm if c.adm is not None else _Admission(c.key, meta(pod).get("uid", ""))
            md = meta(pod)
            claimed = adm.claimed | set(ids)
            done = adm.done + 1
            finished = done >= len(steps)
            now = int(self.clock())
            ann: Dict[str, Optional[str]] = {}
            if pa is None:
                if finished or len(claimed) >= self._pod_request(pod):
                    ann = {ANN_GROUP: format_group(sorted(claimed)), ANN_ASSIGNED: "true", ANN_ASSUME_TIME: str(now)}
            else:
                group = set(pa.group)
                if not claimed <= group:
                    extra = claimed - group
                    spare = sorted(group - claimed, reverse=True)  # GROUP devices no container got yet
                    group = (group - set(spare[:len(extra)])) | claimed
                    log.warning("kubelet allocated %s but pod %s was assumed %s; recording what the kubelet chose",
                                ids, md.get("name"), pa.group)
                    self.metrics.group_overridden.inc()
                complete = claimed >= group
                if sorted(group) != sorted(set(pa.group)) or (complete and not pa.assigned):
                    ann = {ANN_GROUP: format_group(sorted(group)), ANN_ASSIGNED: "true" if complete else "false"}
                    if complete:
                        ann[ANN_ASSUME_TIME] = str(now)
            if ann:
                try:
                    pod = self.api.patch_pod_annotations(md.get("namespace", "default"), md["name"], ann,
                                                         resource_version=md.get("resourceVersion"))
                except Conflict:
                    continue  # someone else touched the pod: re-read and retry
                except Exception as e:  # noqa: BLE001 - the reconcile pass repairs it
                    log.warning("recording allocation %s on %s/%s failed: %s", ids, md.get("namespace"), md.get("name"), e)
            adm.claimed, adm.done = claimed, done
            self._claimed_by = adm
            if finished:
                self._admissions.pop(adm.key, None)
            else:
                self._admissions[adm.key] = adm
            if how != "group" or not finished or len(steps) > 1:
                self.metrics.container_claims.labels(how if how != "group" else ("final" if finished else "partial")).inc()
            return pod
        return None

    def _pod_request(self, pod: dict) -> int:
        try:
            return pod_gpu_request(pod, self._resource_names())
        except ValueError:
            return 0

    def reconcile(self) -> int:
        """Make every GPU pod's ``ALIYUN_COM_GPU_GROUP`` on this node equal the devices the kubelet
        actually gave it (pod-resources ``List``): the annotation is what the extender's view is built
        from, so a swapped pair would let it place a new pod on a device that is in use.  Returns the
        number of pods corrected."""
        sock = self.cfg.pod_resources_socket
        if self.api is None or not self.cfg.node_name or not sock or not os.path.exists(sock):
            return 0
        try:
            truth = list_pod_resources(sock)
        except Exception as e:  # noqa: BLE001 - kubelet restarting: next pass
            log.debug("pod-resources List failed: %s", e)
            return 0
        names = self._resource_names()
        fixed = 0
        pods = self._node_pods(cached=True)
        reported = {}
        for p in pods:
            md = meta(p)
            key = f"{md.get('namespace', 'default')}/{md.get('name')}"
            reported[key] = {int(i) for r in names for i in truth.get(key, {}).get(r, []) if str(i).isascii() and str(i).isdigit()}
        # pod-resources lists app containers and sidecars, not the init containers that have exited,
        # yet the kubelet counts an init container's devices as the pod's until it ends.  Where they
        # went: (1) what this plugin saw allocated together (an admission unit: the calls of one kubelet
        # pod admission, linked by reused devices); (2) after a plugin restart, the GROUPs as written:
        # GROUP devices no pod lists go to the pod listing most of that GROUP, up to its request
        with self._alloc_lock:
            settled = time.monotonic() - self._last_alloc > self.cfg.admission_settle_s
            unit_of = dict(self._unit_of)
        listed = set().union(*reported.values()) if reported else set()
        old = {}
        for p in pods:
            pa = PodAssignment.from_annotations(obj_annotations(p))
            if pa is not None:
                old[pod_key(p)] = set(pa.group)
        orphans: Dict[str, set] = {}
        for g in old.values():
            rest = g - listed
            if not rest:
                continue
            owners = sorted(reported, key=lambda k: (-len(g & reported[k]), k))
            if owners and g & reported[owners[0]]:
                orphans.setdefault(owners[0], set()).update(rest)
        for p in pods:
            md = meta(p)
            key = f"{md.get('namespace', 'default')}/{md.get('name')}"
            ids = set(reported[key])
            if not ids:
                continue  # not admitted yet (or not ours)
            if pod_phase(p) == "Pending" and not settled:
                continue  # the kubelet may be admitting it: its Allocate calls record it
            pa = PodAssignment.from_annotations(obj_annotations(p))
            others = listed - ids
            if all(d in unit_of for d in ids):
                target = set().union(*(unit_of[d] for d in ids)) - others
            else:
                target = ids | set(sorted(orphans.get(key, ()))[:max(0, self._pod_request(p) - len(ids))])
            ids = sorted(target)
            if pa is not None and pa.assigned and ids == sorted(set(pa.group)):
                continue
            ann = {ANN_GROUP: format_group(ids), ANN_ASSIGNED: "true"}
            if pa is None:
                ann[ANN_ASSUME_TIME] = str(int(self.clock()))
            try:
                self.api.patch_pod_annotations(md.get("namespace", "default"), md["name"], ann,
                                               resource_version=md.get("resourceVersion"))
            except Exception as e:  # noqa: BLE001 - conflict or apiserver error: next pass
                log.info("reconciling %s failed (%s); retrying next pass", key, e)
                continue
            fixed += 1
            self.metrics.reconciled.inc()
            log.warning("pod %s: GROUP %s -> %s (kubelet pod-resources)", key, pa.group if pa else None, ids)
            record_event(self.api, p, "GPUAllocationReconciled",
                         f"GROUP {format_group(pa.group) if pa else '-'} -> {format_group(ids)} (kubelet pod-resources)",
                         "Normal", component="gpu-topology-device-plugin", host=self.cfg.node_name)
        return fixed

    # ------------------------------------------------------------------ lifecycle
    def _handlers(self):
        svc = pb.DEVICE_PLUGIN_SERVICE
        h = {}
        for path, (req, res, stream) in pb.METHODS.items():
            if not path.startswith(f"/{svc}/"):
                continue
            name = path.rsplit("/", 1)[1]
            fn = getattr(self, name)
            mk = grpc.unary_stream_rpc_method_handler if stream else grpc.unary_unary_rpc_method_handler
            h[name] = mk(fn, request_deserializer=req.FromString, response_serializer=res.SerializeToString)
        return grpc.method_handlers_generic_handler(svc, h)

    def serve(self) -> None:
        os.makedirs(self.cfg.socket_dir, exist_ok=True)
        try:
            os.unlink(self.cfg.socket_path)
        except FileNotFoundError:
            pass
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=16, thread_name_prefix="devplugin"))
        self._server.add_generic_rpc_handlers((self._handlers(),))
        self._server.add_insecure_port(f"unix://{self.cfg.socket_path}")
        self._server.start()
        log.info("device plugin serving %s on %s", self.cfg.resource_name, self.cfg.socket_path)

    def register(self, timeout: float = 10.0) -> None:
        with grpc.insecure_channel(f"unix://{self.cfg.kubelet_socket}") as ch:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            call = ch.unary_unary(f"/{pb.REGISTRATION_SERVICE}/Register", request_serializer=pb.RegisterRequest.SerializeToString,
                                  response_deserializer=pb.Empty.FromString)
            call(pb.RegisterRequest(version=pb.VERSION, endpoint=self.cfg.socket_name, resource_name=self.cfg.resource_name,
                                    options=pb.DevicePluginOptions(pre_start_required=self.cfg.prestart_validate,
                                                                   get_preferred_allocation_available=True)),
                 timeout=timeout)
        self.registered += 1
        self.metrics.registrations.inc()
        log.info("registered %s with kubelet at %s", self.cfg.resource_name, self.cfg.kubelet_socket)

    def write_cdi_spec(self) -> Optional[str]:
        """(``device_specs == "cdi"``) the CDI spec of the advertised devices -> its path."""
        if self.cfg.device_specs != "cdi":
            return None
        from .cdi import build_spec, write_spec

        path = write_spec(build_spec(self.topology, self.cfg.cdi_kind, self.cfg.dev_root), self.cfg.cdi_dir)
        log.info("CDI spec for %d devices written to %s", self.topology.n, path)
        return path

    def _clear_stale_mark(self) -> None:
        """At start-up, after the node's topology is published: drop a ``<prefix>/probing`` mark the
        previous run left (it marks the node before exiting for a layout change, so the extender
        keeps away until this run has published the new layout)."""
        if self.api is None or not self.cfg.node_name:
            return
        try:
            ann = (self.api.get_node(self.cfg.node_name).get("metadata") or {}).get("annotations") or {}
        except Exception:  # noqa: BLE001 - a mark left in place expires at its deadline
            return
        if self.cfg.contract.probing_key in ann:
            log.info("clearing the probing mark of the previous run (new layout published)")
            self._mark_probing(None)

    def liveness(self, monitor_stall_s: float = 120.0, register_fail_s: float = 300.0) -> Tuple[bool, str]:
        """What ``/healthz`` answers (the DaemonSet's livenessProbe): (ok, reason).  Not alive when the
        gRPC server is down, the monitor loop (health polling, re-registration after a kubelet restart)
        has not passed for ``monitor_stall_s`` — a driver call that never returns wedges it — or
        re-registration has failed for ``register_fail_s``.  The kubelet then restarts the container,
        which starts over from discovery; the pods' devices and annotations are untouched."""
        if not self._started:
            return False, "not started"
        if self._server is None:
            return False, "gRPC server not running"
        now = time.monotonic()
        if self._monitor_beat is not None and now - self._monitor_beat > monitor_stall_s:
            return False, f"monitor loop stalled for {now - self._monitor_beat:.0f}s"
        if self._register_failing_since is not None and now - self._register_failing_since > register_fail_s:
            return False, f"re-registration with the kubelet failing for {now - self._register_failing_since:.0f}s"
        return True, "ok"

    def start(self, register: bool = True) -> None:
        self._stop.clear()
        self.install_guard()
        self.write_cdi_spec()
        self._publish_node()
        self._clear_stale_mark()
        self.serve()
        self._register_required = register
        if register:
            self.register()
        self._started = True
        self._monitor_beat = time.monotonic()
        self._threads = [threading.Thread(target=self._monitor, name="devplugin-monitor", daemon=True)]
        if self.reprobe_fn is not None and (self.cfg.reprobe_interval > 0 or self.event_source is not None):
            # its own thread: a probe takes minutes and must not stall health polling / re-registration
            self._threads.append(threading.Thread(target=self._reprobe_loop, name="devplugin-reprobe", daemon=True))
        if self.event_source is not None:
            self._threads.append(threading.Thread(target=self.event_source.run, args=(self, self._stop),
                                                  name="devplugin-gpu-events", daemon=True))
        for t in self._threads:
            t.start()

    def _reprobe_loop(self) -> None:
        """Every ``reprobe_interval`` s (0 = never), or as soon as a finished GPU reset asks for it (the
        reset may have retrained links) and the node is idle."""
        interval = self.cfg.reprobe_interval if self.cfg.reprobe_interval > 0 else float("inf")
        deadline = time.monotonic() + interval
        while not self._stop.is_set():
            if not self._reprobe_now.is_set() and time.monotonic() < deadline:
                self._reprobe_now.wait(min(1.0, deadline - time.monotonic()))
                continue
            if self._reprobe_now.is_set() and not self.node_idle():
                self._stop.wait(5.0)  # keep the request; retry once the node drains
                continue
            self._reprobe_now.clear()
            deadline = time.monotonic() + interval
            try:
                self.reprobe()
            except Exception as e:
                log.warning("link re-probe failed: %s", e)

    # ------------------------------------------------------------------ GPU events (amdsmi notification)
    def gpu_event(self, index: int, kind: str, message: str = "") -> None:
        """One amdsmi GPU event for device ``index`` (SURVEY.md §5.3 failure detection, between RAS polls):
        ``GPU_PRE_RESET`` holds the device Unhealthy at once (a reset kills every queue on it);
        ``GPU_POST_RESET`` releases the hold — the next RAS pass decides — and asks for a link
        re-measurement once the node is idle; ``VMFAULT`` / ``THERMAL_THROTTLE`` are counted and
        recorded as Node events (a VM fault is a workload's bug, throttling a cooling problem: neither
        takes the device out of service)."""
        if not 0 <= index < self.topology.n:
            return
        self.metrics.gpu_events.labels(kind).inc()
        bdf = self.topology.gpus[index].bdf or "no bdf"
        node = {"kind": "Node", "metadata": {"name": self.cfg.node_name}}
        # the time slices of a GPU (topology/shares.py) are one device: a reset takes all of them
        same = ([g.index for g in self.topology.gpus if g.physical == self.topology.gpus[index].physical]
                if slices_per_gpu(self.topology) > 1 else [index])
        if kind == "GPU_PRE_RESET":
            log.warning("device %d (%s): GPU reset starting: %s", index, bdf, message)
            with self._cond:  # apply_cordon checks and releases holds under this lock
                for i in same:  # a cordoned GPU goes back to its cordon when the reset ends (_cordon_want)
                    self._holds[i] = "GPU reset in progress"
            self.set_health_many({i: False for i in same})
            reason, note = "GPUReset", f"device {index} ({bdf}) is resetting; held Unhealthy"
        elif kind == "GPU_POST_RESET":
            log.warning("device %d (%s): GPU reset finished: %s", index, bdf, message)
            with self._cond:
                for i in same:
                    if i in self._cordon_want:  # cordoned during the reset: the operator's hold replaces it
                        self._holds[i] = self.CORDON_HOLD
                    else:
                        self._holds.pop(i, None)
            if self.health_fn is None:
                self.set_health_many({i: True for i in same if i not in self._holds})
            self._reprobe_now.set()
            reason, note = "GPUResetDone", f"device {index} ({bdf}) finished a reset; links re-measured when idle"
        elif kind == "VMFAULT":
            log.warning("device %d (%s): VM fault: %s", index, bdf, message)
            reason, note = "GPUVMFault", f"device {index} ({bdf}): GPU VM fault: {message[:200]}"
        elif kind == "THERMAL_THROTTLE":
            log.warning("device %d (%s): thermal throttling: %s", index, bdf, message)
            reason, note = "GPUThermalThrottle", f"device {index} ({bdf}) is thermally throttled: {message[:200]}"
        else:
            return
        if self.api is not None and self.cfg.node_name:
            record_event(self.api, node, reason, note, "Normal" if kind == "GPU_POST_RESET" else "Warning",
                         component="gpu-topology-device-plugin", host=self.cfg.node_name)

    def _monitor(self) -> None:
        """Health polling and kubelet restart detection (the kubelet wipes plugin sockets on restart)."""
        next_health = next_reconcile = 0.0
        while not self._stop.wait(0.2):
            self._monitor_beat = time.monotonic()
            # a kubelet restart first: the reconcile below talks to the kubelet's pod-resources socket,
            # which is going away too, and could hold the beat for its RPC timeout before re-registering
            vanished = not os.path.exists(self.cfg.socket_path)
            if not vanished and self.cfg.reconcile_interval > 0 and time.monotonic() >= next_reconcile:
                next_reconcile = time.monotonic() + self.cfg.reconcile_interval
                try:
                    self.reconcile()
                except Exception as e:  # noqa: BLE001
                    log.warning("reconcile failed: %s", e)
            if vanished:
                log.warning("plugin socket %s vanished (kubelet restart?): re-serving and re-registering", self.cfg.socket_path)
                try:
                    if self._server is not None:
                        self._server.stop(grace=0)
                    self.serve()
                    if self._register_required:
                        self.register()
                    self._register_failing_since = None
                except Exception as e:
                    if self._register_failing_since is None:
                        self._register_failing_since = time.monotonic()
                    log.warning("re-registration failed, will retry: %s", e)
            if self.health_fn is not None and time.monotonic() >= next_health:
                next_health = time.monotonic() + self.cfg.health_interval
                try:
                    self.set_health_many({int(idx): bool(ok) and int(idx) not in self._holds
                                          for idx, ok in self.health_fn(self.topology).items()})
                    changed = getattr(self.health_fn, "layout_changed", lambda: None)()
                    if changed:
                        if not self.layout_change.is_set():
                            log.warning("device layout changed (%s): restart required", changed)
                            self.layout_change_reason = changed
                            if self.api is not None and self.cfg.node_name:
                                record_event(self.api, {"kind": "Node", "metadata": {"name": self.cfg.node_name}},
                                             "GPULayoutChanged", f"{changed}; device plugin restarting", "Warning",
                                             component="gpu-topology-device-plugin", host=self.cfg.node_name)
                            self.layout_change.set()
                        continue
                    relink = getattr(self.health_fn, "relink", None)
                    new = relink(self.topology) if relink is not None else None
                    if new is not None:  # a link retrained at another class / went down: republish
                        for g in new.gpus:
                            g.healthy = self._health.get(g.index, True)
                        self.update_topology(new)
                        if self.api is not None and self.cfg.node_name:
                            record_event(self.api, {"kind": "Node", "metadata": {"name": self.cfg.node_name}}, "GPULinkChanged",
                                         f"link class changed for pairs {new.probe.get('relinked')}", "Warning",
                                         component="gpu-topology-device-plugin", host=self.cfg.node_name)
                except Exception as e:
                    log.warning("health check failed: %s", e)

    def stop(self) -> None:
        self._started = False
        self._stop.set()
        with self._cond:
            self._cond.notify_all()
        if self._server is not None:
            self._server.stop(grace=0.5).wait()
            self._server = None
        for t in self._threads:
            t.join(timeout=2)
        try:
            os.unlink(self.cfg.socket_path)
        except FileNotFoundError:
            pass
