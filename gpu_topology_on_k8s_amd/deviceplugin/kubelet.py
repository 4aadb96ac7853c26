"""A fake kubelet device manager speaking the real ``v1beta1`` gRPC protocol (SURVEY.md §4 "fake kubelet").

It serves ``Registration`` on ``<dir>/kubelet.sock``; when a plugin registers it dials the plugin's
endpoint, consumes ``ListAndWatch`` (updating the node's capacity/allocatable in the fake
apiserver, as the real kubelet does — diagram step 2), and on pod admission calls
``GetPreferredAllocation`` + ``Allocate`` the way the kubelet's device manager does: once per
container with that container's count, init containers first, a regular init container's devices
reused by the containers after it (``must_include``).  ``restart()`` wipes the socket directory like
a kubelet restart so plugin re-registration can be tested.

``topology_policy`` / ``topology_scope`` run the kubelet's Topology Manager in front of the device
manager (``--topology-manager-policy`` / ``--topology-manager-scope``): NUMA hints from the devices'
``TopologyInfo``, merged by the policy, admission refused with ``TopologyAffinityError``, and each
container's devices drawn from the hinted NUMA nodes first (the device manager's ``filterByAffinity``).
The device manager is the only hint provider modelled (no CPU or memory manager).
"""
from __future__ import annotations

import glob
import logging
import os
import threading
import time
from concurrent import futures
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import grpc

from ..k8s.objects import meta, pod_device_steps, pod_gpu_request, pod_key
from .podresources import build_response, pod_resources_handler
from . import proto as pb

log = logging.getLogger(__name__)

__all__ = ["FakeKubelet", "AdmissionError", "TOPOLOGY_POLICIES"]

TOPOLOGY_POLICIES = ("none", "best-effort", "restricted", "single-numa-node")


class AdmissionError(RuntimeError):
    pass


@dataclass
class _Plugin:
    resource: str
    endpoint: str
    channel: grpc.Channel
    options: object
    devices: Dict[str, str] = field(default_factory=dict)  # id -> health
    numa: Dict[str, Tuple[int, ...]] = field(default_factory=dict)  # id -> NUMA nodes of its TopologyInfo
    ready: threading.Event = field(default_factory=threading.Event)
    thread: Optional[threading.Thread] = None


class FakeKubelet:
    def __init__(self, socket_dir: str, node_name: str = "", api=None, pod_resources_socket: Optional[str] = None,
                 cdi_dir: Optional[str] = None, topology_policy: str = "none", topology_scope: str = "container"):
        if topology_policy not in TOPOLOGY_POLICIES or topology_scope not in ("container", "pod"):
            raise ValueError(f"topology manager policy/scope {topology_policy}/{topology_scope} not supported")
        self.topology_policy = topology_policy
        self.topology_scope = topology_scope
        self.socket_dir = socket_dir
        # a CDI-enabled runtime resolves Allocate's cdi_devices against the specs in this directory
        self.cdi_dir = cdi_dir
        # the pod-resources API (v1 PodResourcesLister.List) lives in its own directory on a real
        # node (/var/lib/kubelet/pod-resources/kubelet.sock); here a subdirectory of socket_dir
        self.pod_resources_socket = pod_resources_socket or os.path.join(socket_dir, "pod-resources", "kubelet.sock")
        self.node_name = node_name
        self.api = api
        self.plugins: Dict[str, _Plugin] = {}
        self.allocated: Dict[str, Dict[str, Tuple[str, ...]]] = {}  # resource -> pod key -> ids (every container's)
        # resource -> pod key -> [(container, kind, ids)] in admission order (pod-resources reports these)
        self.containers: Dict[str, Dict[str, List[Tuple[str, str, Tuple[str, ...]]]]] = {}
        self.allocate_calls: List[Tuple[str, str, Tuple[str, ...]]] = []  # (pod key, container, ids) per Allocate RPC
        self.preferred_calls: List[Tuple[List[str], int]] = []  # (must_include, size) per GetPreferredAllocation RPC
        self.responses: Dict[str, object] = {}  # pod key -> AllocateResponse
        self.rejected: List[Tuple[str, str]] = []  # (pod key, reason) of pods whose admission failed
        self._server: Optional[grpc.Server] = None
        self._lock = threading.RLock()
        self._stop = threading.Event()

    @property
    def socket(self) -> str:
        return os.path.join(self.socket_dir, "kubelet.sock")

    # ------------------------------------------------------------------ Registration service
    def Register(self, request, context):
        if request.version != pb.VERSION:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"unsupported version {request.version}")
        ep = os.path.join(self.socket_dir, request.endpoint)
        ch = grpc.insecure_channel(f"unix://{ep}")
        old = self.plugins.get(request.resource_name)
        p = _Plugin(resource=request.resource_name, endpoint=ep, channel=ch, options=request.options)
        with self._lock:
            self.plugins[request.resource_name] = p
            self.allocated.setdefault(request.resource_name, {})
        if old is not None:
            old.channel.close()
        p.thread = threading.Thread(target=self._watch, args=(p,), name=f"kubelet-law-{request.resource_name}", daemon=True)
        p.thread.start()
        return pb.Empty()

    def _stub(self, p: _Plugin, method: str):
        req, res, stream = pb.METHODS[f"/{pb.DEVICE_PLUGIN_SERVICE}/{method}"]
        mk = p.channel.unary_stream if stream else p.channel.unary_unary
        return mk(f"/{pb.DEVICE_PLUGIN_SERVICE}/{method}", request_serializer=req.SerializeToString,
                  response_deserializer=res.FromString)

    def _watch(self, p: _Plugin) -> None:
        try:
            for resp in self._stub(p, "ListAndWatch")(pb.Empty()):
                with self._lock:
                    p.devices = {d.ID: d.health for d in resp.devices}
                    p.numa = {d.ID: tuple(int(n.ID) for n in d.topology.nodes) for d in resp.devices}
                p.ready.set()
                self._update_capacity(p)
                if self._stop.is_set():
                    break
        except grpc.RpcError as e:
            if not self._stop.is_set():
                log.info("ListAndWatch for %s ended: %s", p.resource, e.code())

    def _update_capacity(self, p: _Plugin) -> None:
        if self.api is None or not self.node_name or not hasattr(self.api, "update_node_status"):
            return
        healthy = sum(1 for h in p.devices.values() if h == pb.HEALTHY)
        try:
            self.api.update_node_status(self.node_name, {p.resource: str(len(p.devices))}, {p.resource: str(healthy)})
        except Exception as e:  # pragma: no cover
            log.warning("capacity update failed: %s", e)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        os.makedirs(self.socket_dir, exist_ok=True)
        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        self._stop.clear()
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=4, thread_name_prefix="kubelet"))
        h = grpc.unary_unary_rpc_method_handler(self.Register, request_deserializer=pb.RegisterRequest.FromString,
                                                response_serializer=pb.Empty.SerializeToString)
        self._server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(pb.REGISTRATION_SERVICE, {"Register": h}),
                                               pod_resources_handler(self.list_pod_resources)))
        self._server.add_insecure_port(f"unix://{self.socket}")
        os.makedirs(os.path.dirname(self.pod_resources_socket), exist_ok=True)
        try:
            os.unlink(self.pod_resources_socket)
        except FileNotFoundError:
            pass
        self._server.add_insecure_port(f"unix://{self.pod_resources_socket}")
        self._server.start()

    def list_pod_resources(self):
        """What the device manager reports (PodResourcesLister.List): per app container and sidecar its
        devices.  Regular init containers are not listed (they have exited), so a pod whose init
        container held more devices than its app containers shows fewer devices than it holds."""
        with self._lock:
            rows = []
            for res, per in self.allocated.items():
                for key, ids in per.items():
                    cs = self.containers.get(res, {}).get(key)
                    if cs is None:
                        rows.append((key, "main", res, list(ids)))
                        continue
                    rows += [(key, name, res, list(cids)) for name, kind, cids in cs if kind != "init"]
        return build_response(rows)

    def stop(self) -> None:
        self._stop.set()
        if self._server is not None:
            self._server.stop(grace=0).wait()
            self._server = None
        for p in list(self.plugins.values()):
            p.channel.close()

    def restart(self) -> None:
        """Like a kubelet restart: stop, wipe every socket in the directory, start again."""
        self.stop()
        for s in glob.glob(os.path.join(self.socket_dir, "*.sock")):
            os.unlink(s)
        with self._lock:
            self.plugins.clear()
        self.start()

    def restart_container(self, key: str, container: str, resource: Optional[str] = None) -> Tuple[str, ...]:
        """A container of an admitted pod restarts (a crash, a liveness failure): like the kubelet, the
        device manager hands it the devices it already holds.  There is no GetPreferredAllocation and no
        Allocate; only PreStartContainer runs again when the plugin asks for it, and its failure fails
        this start (the kubelet backs off and retries).  Returns the container's device ids."""
        resource = resource or next(iter(self.plugins))
        p = self.plugins[resource]
        with self._lock:
            held = [ids for name, _kind, ids in self.containers.get(resource, {}).get(key, ()) if name == container]
        if not held:
            raise KeyError(f"{key}: no container {container!r} holding {resource}")
        ids = held[0]
        if getattr(p.options, "pre_start_required", False):
            try:
                self._stub(p, "PreStartContainer")(pb.PreStartContainerRequest(devices_ids=list(ids)), timeout=300)
            except grpc.RpcError as e:
                raise AdmissionError(f"PreStartContainer failed: {e.details()}") from e
        return ids

    def wait_for(self, resource: str, timeout: float = 10.0) -> _Plugin:
        t0 = time.time()
        while time.time() - t0 < timeout:
            p = self.plugins.get(resource)
            if p is not None and p.ready.wait(timeout=0.05):
                return p
            time.sleep(0.02)
        raise TimeoutError(f"plugin for {resource} did not register/advertise within {timeout}s")

    # ------------------------------------------------------------------ device manager
    def options(self, resource: str):
        return self._stub(self.plugins[resource], "GetDevicePluginOptions")(pb.Empty(), timeout=5)

    def available(self, resource: str) -> List[str]:
        p = self.plugins[resource]
        with self._lock:
            used = {i for ids in self.allocated.get(resource, {}).values() for i in ids}
            return sorted((d for d, h in p.devices.items() if h == pb.HEALTHY and d not in used), key=int)

    def _reject(self, pod: dict, msg: str, reason: str = "UnexpectedAdmissionError") -> AdmissionError:
        """Pod admission failed: like the real kubelet, the pod is terminal (``Failed``, reason
        ``UnexpectedAdmissionError``, or ``TopologyAffinityError`` from the Topology Manager) and is
        never retried on this node; a bare pod is lost."""
        self.rejected.append((pod_key(pod), msg))
        if self.api is not None and hasattr(self.api, "set_pod_phase"):
            md = meta(pod)
            try:
                self.api.set_pod_phase(md.get("namespace", "default"), md["name"], "Failed", reason=reason, message=msg)
            except Exception:  # pragma: no cover
                pass
        return AdmissionError(f"{reason}: {msg}")

    # ------------------------------------------------------------------ topology manager
    # NUMA sets are bitmasks (bit i = NUMA node i), as in the kubelet's bitmask package.
    def _numa_nodes(self, p: _Plugin) -> List[int]:
        return sorted({n for ns in p.numa.values() for n in ns})

    def _device_mask(self, p: _Plugin, d: str) -> int:
        m = 0
        for n in p.numa.get(d, ()):
            m |= 1 << n
        return m

    @staticmethod
    def _iterate_masks(nodes: List[int]):
        """``bitmask.IterateBitMasks``: every combination of ``nodes``, one bit first, in order."""
        def rec(rest, acc, size):
            if len(acc) == size:
                yield sum(1 << b for b in acc)
                return
            for i in range(len(rest)):
                yield from rec(rest[i + 1:], acc + [rest[i]], size)
        for size in range(1, len(nodes) + 1):
            yield from rec(nodes, [], size)

    def _generate_hints(self, p: _Plugin, available: set, reusable: set, request: int) -> Optional[List[Tuple[int, bool]]]:
        """``generateDeviceTopologyHints``: None = the resource has no topology (no preference); [] = no
        NUMA combination can hold the request."""
        nodes = self._numa_nodes(p)
        if not nodes:
            return None
        if len(available | reusable) < request:
            return []
        min_affinity = len(nodes)
        hints: List[Tuple[int, bool]] = []
        for mask in self._iterate_masks(nodes):
            in_mask = sum(1 for d in p.devices if self._device_mask(p, d) & mask)
            if in_mask >= request and bin(mask).count("1") < min_affinity:
                min_affinity = bin(mask).count("1")
            matching = 0
            fits = True
            for d in reusable:
                dm = self._device_mask(p, d)
                if not dm:
                    continue
                if not dm & mask:
                    fits = False
                    break
                matching += 1
            if not fits:
                continue
            matching += sum(1 for d in available if self._device_mask(p, d) & mask)
            if matching >= request:
                hints.append((mask, False))
        return [(m, bin(m).count("1") == min_affinity) for m, _ in hints]

    def _merge(self, p: _Plugin, hints: Optional[List[Tuple[int, bool]]]) -> Tuple[Optional[int], bool]:
        """The policy's ``Merge`` with the device manager as the only provider -> (mask or None, admit)."""
        nodes = self._numa_nodes(p)
        default = sum(1 << n for n in nodes)
        if hints is None:
            return None, True
        if self.topology_policy == "single-numa-node":
            hints = [(m, pref) for m, pref in hints if bin(m).count("1") == 1 and pref]
        best_mask, best_pref = default, False  # mergeFilteredHints starts from {default, false}
        for m, pref in hints:
            if pref and not best_pref:
                best_mask, best_pref = m, pref
                continue
            if best_pref and not pref:
                continue
            cm, cb = bin(m).count("1"), bin(best_mask).count("1")
            narrower = cm < cb or (cm == cb and m < best_mask)  # IsNarrowerThan: equal widths compare as integers
            if narrower:
                best_mask, best_pref = m, pref
        if self.topology_policy == "single-numa-node" and best_mask == default:
            best_mask = None
        admit = self.topology_policy == "best-effort" or best_pref
        return best_mask, admit

    def _hint(self, p: _Plugin, pod: dict, request: int, available: set, reusable: set) -> Optional[int]:
        """Admit one hint request or reject the pod (``TopologyAffinityError``)."""
        mask, admit = self._merge(p, self._generate_hints(p, available, reusable, request))
        if not admit:
            raise self._reject(pod, f"Resources cannot be allocated with Topology locality (policy {self.topology_policy}, "
                                    f"scope {self.topology_scope}, {request} devices)", reason="TopologyAffinityError")
        return mask

    def _devices_to_allocate(self, p: _Plugin, resource: str, required: int, in_use: set, reusable: List[str],
                             hint: Optional[int] = None) -> List[str]:
        """``devicesToAllocate`` of the kubelet device manager for one container: devices an init
        container of the pod handed on come first.  With a Topology Manager hint (``filterByAffinity``)
        the free devices on the hinted NUMA nodes are ``aligned``: if the container needs fewer than
        that, the plugin's ``GetPreferredAllocation`` is asked with ``aligned ∪ reused``; otherwise it
        gets every aligned device and the plugin is asked with ``available ∪ allocated`` for the rest.
        Without a hint it is asked with ``available ∪ reused``.  ``must_include`` is what the container
        holds already, the size its full count; the answer ∩ the offered devices fills the request,
        then the lowest free ids (Go's set order is unspecified)."""
        allocated: List[str] = []

        def allocate_remaining_from(devices) -> bool:
            for d in sorted(devices, key=int):
                if len(allocated) == required:
                    break
                if d not in allocated:
                    allocated.append(d)
            return len(allocated) == required

        if allocate_remaining_from(sorted(reusable, key=int)):
            return allocated
        avail = [d for d in self.available(resource) if d not in in_use and d not in allocated]
        needed = required - len(allocated)
        if len(avail) < needed:
            raise ValueError(f"requested number of devices unavailable for {resource}. Requested: {required}, "
                             f"Available: {len(avail) + len(allocated)}")
        aligned = [d for d in avail if hint is not None and self._device_mask(p, d) & hint]
        unaligned = [d for d in avail if d not in aligned]

        def preferred(offered) -> List[str]:
            if not getattr(p.options, "get_preferred_allocation_available", False):
                return []
            req = pb.PreferredAllocationRequest()
            req.container_requests.add(available_deviceIDs=sorted(set(offered) | set(allocated), key=int),
                                       must_include_deviceIDs=list(allocated), allocation_size=required)
            self.preferred_calls.append((list(allocated), required))
            resp = self._stub(p, "GetPreferredAllocation")(req, timeout=5)
            return [d for d in resp.container_responses[0].deviceIDs if d in offered]

        if needed < len(aligned):
            if allocate_remaining_from(preferred(aligned)) or allocate_remaining_from(aligned):
                return allocated
            raise ValueError(f"unexpectedly allocated less resources than required. Requested: {required}")
        if allocate_remaining_from(aligned):
            return allocated
        if allocate_remaining_from(preferred(avail)):
            return allocated
        allocate_remaining_from(unaligned)
        return allocated

    def admit(self, pod: dict, resource: str, allocate_timeout: float = 10.0):
        """Admit ``pod`` the way the kubelet's device manager does (``ManagerImpl.Allocate``): once per
        container that requests ``resource`` — init containers first, then the app containers — one
        ``GetPreferredAllocation`` (when the plugin offers it and reused devices do not cover the
        request) and one ``Allocate`` with that container's devices.  A regular init container's
        devices are reused by the containers after it; a sidecar's are not.  Any error of either call,
        or too few devices, rejects the pod for good (:meth:`_reject`); a missing device node or a
        failed PreStartContainer only fails the container start (retried by the kubelet), so the pod
        stays Pending.  Returns one AllocateResponse holding every container's response, in order."""
        key = pod_key(pod)
        p = self.plugins.get(resource)
        names = [resource] + [r for r in self.plugins if r != resource]
        steps = pod_device_steps(pod, names)
        if not steps:
            return None
        if p is None:
            raise self._reject(pod, f"no device plugin registered for {resource}")
        with self._lock:
            reuse: List[str] = []  # devicesToReuse[pod]
            pod_ids: List[str] = []  # every device the pod holds (the device manager's podDevices)
            per_container: List[Tuple[str, str, Tuple[str, ...]]] = []
            resp = pb.AllocateResponse()
            tm = self.topology_policy != "none"
            hint: Optional[int] = None
            if tm and self.topology_scope == "pod":
                hint = self._hint(p, pod, pod_gpu_request(pod, [resource]), set(self.available(resource)), set())
            try:
                for cname, n, kind in steps:
                    if tm and self.topology_scope == "container":
                        free = {d for d in self.available(resource) if d not in pod_ids}
                        hint = self._hint(p, pod, n, free, set(reuse))
                    try:
                        chosen = self._devices_to_allocate(p, resource, n, set(pod_ids), reuse, hint)
                    except ValueError as e:
                        raise self._reject(pod, str(e)) from e
                    areq = pb.AllocateRequest()
                    areq.container_requests.add(devices_ids=chosen)
                    self.allocate_calls.append((key, cname, tuple(chosen)))
                    r = self._stub(p, "Allocate")(areq, timeout=allocate_timeout)
                    resp.container_responses.extend(r.container_responses)
                    pod_ids += [d for d in chosen if d not in pod_ids]
                    per_container.append((cname, kind, tuple(chosen)))
                    if kind == "init":
                        reuse += [d for d in chosen if d not in reuse]
                    else:  # an app container or a sidecar keeps what it got
                        reuse = [d for d in reuse if d not in chosen]
            except grpc.RpcError as e:
                raise self._reject(pod, f"device plugin call failed: {e.code()}: {e.details()}") from e
            # what containerd does next: every DeviceSpec must name a device node that exists on the
            # host, or the container is never created (BASELINE config 1 on a kind node)
            missing = [d.host_path for c in resp.container_responses for d in c.devices if not os.path.exists(d.host_path)]
            # bind-mount sources must exist too (the runtime fails the container otherwise)
            missing += [m.host_path for c in resp.container_responses for m in c.mounts if not os.path.exists(m.host_path)]
            for c in resp.container_responses:
                for cd in c.cdi_devices:
                    missing += self._cdi_missing(cd.name)
            if missing:
                raise AdmissionError(f"CreateContainerError: device nodes do not exist on the node: {missing}")
            if getattr(p.options, "pre_start_required", False):
                # the kubelet calls PreStartContainer per container before starting it; an error
                # there fails the container start
                for _, _, ids in per_container:
                    try:
                        self._stub(p, "PreStartContainer")(pb.PreStartContainerRequest(devices_ids=list(ids)), timeout=300)
                    except grpc.RpcError as e:
                        raise AdmissionError(f"PreStartContainer failed: {e.details()}") from e
            self.allocated[resource][key] = tuple(sorted(pod_ids, key=int))
            self.containers.setdefault(resource, {})[key] = per_container
            self.responses[key] = resp
        if self.api is not None and hasattr(self.api, "set_pod_phase"):
            md = meta(pod)
            try:
                self.api.set_pod_phase(md.get("namespace", "default"), md["name"], "Running")
            except Exception:  # pragma: no cover
                pass
        return resp

    def _cdi_missing(self, name: str) -> List[str]:
        """What a CDI runtime would fail on for device ``name`` (``vendor/class=dev``): no spec of that
        kind, no such device, or a device node the spec names that is absent on the host."""
        import glob
        import json

        kind, _, dev = name.partition("=")
        for path in sorted(glob.glob(os.path.join(self.cdi_dir or "/nonexistent", "*.json"))):
            with open(path) as f:
                spec = json.load(f)
            if spec.get("kind") != kind:
                continue
            for d in spec.get("devices", []):
                if d.get("name") == dev:
                    nodes = list(d.get("containerEdits", {}).get("deviceNodes", []))
                    nodes += spec.get("containerEdits", {}).get("deviceNodes", [])
                    return [n.get("hostPath") or n["path"] for n in nodes if not os.path.exists(n.get("hostPath") or n["path"])]
            return [f"CDI device {name} not in {path}"]
        return [f"unresolvable CDI device {name}"]

    def release(self, pod: dict) -> None:
        key = pod_key(pod)
        with self._lock:
            for res in self.allocated.values():
                res.pop(key, None)
            for per in self.containers.values():
                per.pop(key, None)


def _bits(mask: int) -> List[int]:
    return [i for i in range(mask.bit_length()) if mask >> i & 1]
