"""In-process Kubernetes cluster: fake apiserver + mini kube-scheduler + extender (HTTP) + per-node
fake kubelet and real device plugin over gRPC (SURVEY.md §4 "Integration: cluster in a process",
§7.1 step 8).

It drives the reference's 7-step flow end to end (``imgs/gpu_topology_on_k8s.png``):
  1-2. each node's device plugin registers with its kubelet, ListAndWatch -> node capacity;
       the plugin publishes the topology annotations (design.md:76-86);
  3.   the mini scheduler filters by extended-resource fit (the default scheduler's job,
       design.md:117), then POSTs ``{prefix}/sort`` to the extender and picks the best node;
  4-5. it POSTs ``{prefix}/bind``; the extender writes GROUP/ASSIGNED/ASSUME_TIME and binds;
  6-7. the node's kubelet admits the pod: GetPreferredAllocation + Allocate over gRPC; the plugin
       flips ASSIGNED=true and returns the device nodes.
Used for BASELINE config 1 (2 fake GPUs, 1-GPU pod), config 4 (two concurrent 4-GPU pods),
restart recovery, fault injection and the scheduling-latency benchmark.
"""
from __future__ import annotations

import asyncio
import copy
import logging
import os
import shutil
import tempfile
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import http.client
import json
from urllib.parse import urlsplit
from aiohttp import web

from ..deviceplugin import DevicePluginServer, FakeKubelet, PluginConfig, placeholder_dev_tree
from ..deviceplugin.kubelet import AdmissionError
from ..extender import ExtenderConfig, TopologyExtender
from ..extender.server import DEFAULT_PREFIX, make_app
from ..k8s import Contract, FakeAPIServer, PodAssignment
from ..k8s.objects import annotations as obj_annotations
from ..k8s.objects import make_node, make_pod, meta, pod_gpu_request, pod_is_terminal, pod_key, pod_node
from ..placement import PlacementPolicy
from ..topology.model import Topology
from ..topology.shares import slices_per_gpu

log = logging.getLogger(__name__)

__all__ = ["SimCluster", "ScheduleResult", "HttpExtender"]


class _ExtenderClient:
    """kube-scheduler's side of the extender protocol: JSON POSTs over a keep-alive connection per
    calling thread (the Go client reuses its connections too; ``requests`` added ~1.5 ms per verb to
    every measured scheduling time).  A connection the server closed while idle (extender restart)
    is re-opened and the request re-sent once."""

    def __init__(self):
        self._tls = threading.local()
        self._all: List[http.client.HTTPConnection] = []
        self._lock = threading.Lock()

    @property
    def _conn(self) -> Optional[http.client.HTTPConnection]:
        return getattr(self._tls, "conn", None)

    @_conn.setter
    def _conn(self, c: Optional[http.client.HTTPConnection]) -> None:
        self._tls.conn = c
        if c is not None:
            with self._lock:
                self._all.append(c)

    @property
    def _base(self) -> str:
        return getattr(self._tls, "base", "")

    @_base.setter
    def _base(self, b: str) -> None:
        self._tls.base = b

    def post(self, url: str, body: dict, timeout: float = 30.0):
        u = urlsplit(url)
        base = f"{u.hostname}:{u.port}"
        data = json.dumps(body).encode()
        for attempt in (0, 1):
            if self._conn is None or base != self._base:
                self._drop()
                self._conn, self._base = http.client.HTTPConnection(u.hostname, u.port, timeout=timeout), base
            try:
                self._conn.request("POST", u.path, data, {"Content-Type": "application/json"})
                r = self._conn.getresponse()
                payload = r.read()
            except (http.client.RemoteDisconnected, http.client.BadStatusLine, ConnectionError):
                self._drop()
                if attempt:
                    raise
                continue
            if r.status >= 400:
                raise RuntimeError(f"extender {u.path}: HTTP {r.status}: {payload[:200]!r}")
            return json.loads(payload)

    def _drop(self) -> None:
        c = self._conn
        if c is not None:
            c.close()
            self._tls.conn = None

    def close(self) -> None:
        with self._lock:
            conns, self._all = self._all, []
        for c in conns:
            c.close()
        self._tls.conn = None


class HttpExtender:
    """Run the aiohttp extender app on 127.0.0.1:<ephemeral> in a background event-loop thread."""

    def __init__(self, ext: TopologyExtender, prefix: str = DEFAULT_PREFIX):
        self.ext = ext
        self.prefix = prefix
        self.port = 0
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._runner: Optional[web.AppRunner] = None
        self._ready = threading.Event()
        self._thread: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}{self.prefix}"

    def start(self) -> None:
        def run():
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)

            async def up():
                self._runner = web.AppRunner(make_app(self.ext, self.prefix), access_log=None)
                await self._runner.setup()
                site = web.TCPSite(self._runner, "127.0.0.1", 0)
                await site.start()
                self.port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]

            self._loop.run_until_complete(up())
            self._ready.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, name="sim-extender", daemon=True)
        self._thread.start()
        if not self._ready.wait(10):
            raise RuntimeError("extender HTTP server did not start")

    def stop(self) -> None:
        if self._loop is None:
            return

        async def down():
            if self._runner is not None:
                await self._runner.cleanup()

        asyncio.run_coroutine_threadsafe(down(), self._loop).result(10)
        self._loop.call_soon_threadsafe(self._loop.stop)
        if self._thread is not None:
            self._thread.join(5)
        self._loop = None


@dataclass
class ScheduleResult:
    pod: str
    node: Optional[str]
    devices: Tuple[int, ...] = ()
    score: int = 0
    error: str = ""
    sched_ms: float = 0.0  # filter + sort + bind (the paper's "scheduling time", Fig. 10)
    admit_ms: float = 0.0  # kubelet GetPreferredAllocation + Allocate
    allocated: Tuple[int, ...] = ()


@dataclass
class _Node:
    name: str
    topology: Topology
    sockdir: str
    kubelet: FakeKubelet
    plugin: DevicePluginServer
    resource: str = ""  # the extended resource its plugin advertises (slices on a time-sliced node)


class SimCluster:
    def __init__(self, nodes: Dict[str, Topology], resource: str = "amd.com/gpu", policy_name: str = "exact",
                 policy: PlacementPolicy = PlacementPolicy(), assume_ttl: float = 300.0, use_filter: bool = True,
                 node_labels: Optional[Dict[str, Dict[str, str]]] = None, device_specs: str = "strict",
                 prestart_validate: bool = False, validate_fn=None, reconcile_interval: float = 0.0,
                 informer: bool = False, share_guard: str = "preload", rbac: bool = False,
                 topology_manager=None, publish_topology_manager: bool = True, replicas: int = 1):
        self.resource = resource
        # extender replicas (kube-scheduler HA: one extender per control-plane node, each with its own
        # cache); the mini scheduler sends consecutive pods to them in turn
        self.replicas = max(1, int(replicas))
        self._extra: List[Tuple[TopologyExtender, "HttpExtender", object]] = []
        self._turn = 0
        # the kubelets' Topology Manager (placement/numa_align.TopologyManager, one for every node or a
        # dict per node); the plugins publish it unless `publish_topology_manager` is off (an operator
        # who did not tell the plugin: the extender then places as if the policy were none)
        self.topology_manager = topology_manager
        self.publish_topology_manager = publish_topology_manager
        # every component talks to the apiserver as its deploy ServiceAccount (k8s/rbac.py): the
        # plugins with their node-name claim and the own-node admission policy, the extender with its
        # ledger Role; the fake kubelet and the mini scheduler keep full access
        self.rbac = rbac
        self.denied: List[str] = []
        # drive the extender's cache by LIST+WATCH (production mode) instead of a LIST per request
        self.use_informer = informer
        self.informer = None
        # the plugins' pod-resources reconcile loop (0 = only when reconcile() is called: deterministic tests)
        self.reconcile_interval = reconcile_interval
        self.device_specs = device_specs
        self.share_guard = share_guard  # time-sliced nodes: the vGPU guard mounted into partial-GPU pods
        self.prestart_validate = prestart_validate
        self.validate_fn = validate_fn
        self.contract = Contract(resource_name=resource)
        self.api = FakeAPIServer()
        self.ext_cfg = ExtenderConfig(contract=self.contract, policy_name=policy_name, policy=policy, assume_ttl=assume_ttl,
                                      resync_s=0.0)
        self.use_filter = use_filter
        self._root = tempfile.mkdtemp(prefix="gtksim", dir="/tmp")
        self.nodes: Dict[str, _Node] = {}
        self._topologies = dict(nodes)
        self._labels = node_labels or {}
        self.extender: Optional[TopologyExtender] = None
        self.http: Optional[HttpExtender] = None
        self._client = _ExtenderClient()
        self.history: List[ScheduleResult] = []
        self._plugin_args: Dict[str, tuple] = {}

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "SimCluster":
        for i, (name, topo) in enumerate(self._topologies.items()):
            self.api.create_node(make_node(name, labels=self._labels.get(name)))
            sockdir = os.path.join(self._root, f"n{i}")
            tm = self.topology_manager.get(name) if isinstance(self.topology_manager, dict) else self.topology_manager
            kubelet = FakeKubelet(sockdir, node_name=name, api=self.api, topology_policy=tm.policy if tm else "none",
                                  topology_scope=tm.scope if tm else "container")
            kubelet.start()
            if self.device_specs == "strict":  # a node with (placeholder) ROCm device nodes
                dev_root = placeholder_dev_tree(os.path.join(self._root, f"dev{i}"), topo)
            else:  # a kind node: no /dev/kfd, no render nodes
                dev_root = os.path.join(self._root, f"dev{i}")
                os.makedirs(dev_root, exist_ok=True)
            # a time-sliced node is its own pool: its plugin advertises the slice resource (as the
            # daemon does with --time-slices), and amd.com/gpu means whole GPUs everywhere
            res = self.contract.slice_resource if slices_per_gpu(topo) > 1 else self.resource
            self._plugin_args[name] = (i, copy.deepcopy(topo), sockdir, dev_root, kubelet, res, tm)  # as discovered
            plugin = self._make_plugin(name, topo)
            plugin.start()
            kubelet.wait_for(res)
            self.nodes[name] = _Node(name, topo, sockdir, kubelet, plugin, res)
        self.start_extender()
        return self

    def _make_plugin(self, name: str, topo: Optional[Topology] = None) -> DevicePluginServer:
        """The node's plugin; a restarted one re-discovers the node (a pristine copy of its topology)."""
        i, pristine, sockdir, dev_root, kubelet, res, tm = self._plugin_args[name]
        return DevicePluginServer(topo if topo is not None else copy.deepcopy(pristine), PluginConfig(
            resource_name=res, socket_dir=sockdir, node_name=name, contract=self.contract, dev_root=dev_root,
            device_specs=self.device_specs, prestart_validate=self.prestart_validate,
            pod_resources_socket=kubelet.pod_resources_socket, reconcile_interval=self.reconcile_interval,
            share_guard=self.share_guard, guard_dir=os.path.join(self._root, f"vgpu{i}"),
            topology_manager=tm if self.publish_topology_manager else None),
            api=self._as("plugin", name), validate_fn=self.validate_fn)

    def restart_plugin(self, name: str) -> None:
        """The node's device plugin process restarts: a new one with no memory of admissions, which
        reads its node (the operator's cordon) before serving, as the daemon does, and re-registers."""
        n = self.nodes[name]
        n.plugin.stop()
        plugin = self._make_plugin(name)
        plugin.poll_node()
        plugin.start()
        n.kubelet.wait_for(n.resource)
        n.plugin = plugin

    def _as(self, who: str, node: str = ""):
        """The apiserver as the deploy ServiceAccount of ``who`` (plugin / extender) sees it."""
        if not self.rbac:
            return self.api
        import yaml

        from ..config import EXTENDER_SA, NAMESPACE, PLUGIN_SA, render_manifests
        from ..k8s.rbac import RBACView, identities_from_manifests, sa_username

        ids = identities_from_manifests(yaml.safe_load_all(render_manifests()))
        view = RBACView(self.api, ids[sa_username(NAMESPACE, PLUGIN_SA if who == "plugin" else EXTENDER_SA)], node_name=node)
        view.denied = self.denied  # one shared log of refusals
        return view

    def start_extender(self) -> None:
        self.extender, self.http, self.informer = self._new_replica()
        self._extra = [self._new_replica() for _ in range(self.replicas - 1)]

    @property
    def extenders(self) -> List[TopologyExtender]:
        return [self.extender] + [e for e, _, _ in self._extra]

    def _new_replica(self):
        ext = TopologyExtender(self._as("extender"), self.ext_cfg)
        inf = None
        if self.use_informer:
            inf = ext.cache.make_informer(watch_timeout=5.0, backoff=0.1, page_size=50)
            inf.start()
            inf.wait_synced(10.0)
        http = HttpExtender(ext)
        http.start()
        return ext, http, inf

    def _stop_extender(self) -> None:
        if self.http is not None:
            self.http.stop()
            self.http = None
        if self.informer is not None:
            self.informer.stop()
            self.informer = None
        for _, http, inf in self._extra:
            http.stop()
            if inf is not None:
                inf.stop()
        self._extra = []

    def restart_extender(self) -> None:
        """Stateless restart: the new process rebuilds from annotations."""
        self._stop_extender()
        self.start_extender()

    def stop(self) -> None:
        self._client.close()
        self._stop_extender()
        for n in self.nodes.values():
            n.plugin.stop()
            n.kubelet.stop()
        shutil.rmtree(self._root, ignore_errors=True)

    def __enter__(self) -> "SimCluster":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()

    # ------------------------------------------------------------------ workload
    def submit(self, name: str, gpus: int, namespace: str = "default", slices: bool = False, **kw) -> dict:
        """A pod requesting ``gpus`` whole GPUs, or (``slices``) that many time slices."""
        res = self.contract.slice_resource if slices else self.resource
        return self.api.create_pod(make_pod(name, gpus=gpus, namespace=namespace, resource=res, **kw))

    def pod_resource(self, pod: dict) -> str:
        """The pool a pod draws from: the slice resource if it requests slices, else whole GPUs."""
        return self.contract.slice_resource if pod_gpu_request(pod, [self.contract.slice_resource]) else self.resource

    def complete(self, name: str, namespace: str = "default", phase: str = "Succeeded") -> None:
        pod = self.api.get_pod(namespace, name)
        self.api.set_pod_phase(namespace, name, phase)
        n = self.nodes.get(pod_node(pod))
        if n is not None:
            n.kubelet.release(pod)

    def delete(self, name: str, namespace: str = "default") -> None:
        pod = self.api.get_pod(namespace, name)
        self.api.delete_pod(namespace, name)
        n = self.nodes.get(pod_node(pod))
        if n is not None:
            n.kubelet.release(pod)

    # ------------------------------------------------------------------ mini kube-scheduler
    def _fits(self, pod: dict) -> List[str]:
        """Default NodeResourcesFit on the extended resource the pod requests (design.md:117)."""
        res = self.pod_resource(pod)
        k = pod_gpu_request(pod, [res])
        pods = self.api.list_pods()
        out = []
        for node in self.api.list_nodes():
            name = meta(node)["name"]
            alloc = int(float(((node.get("status") or {}).get("allocatable") or {}).get(res, 0)))
            used = sum(pod_gpu_request(p, [res]) for p in pods if pod_node(p) == name and not pod_is_terminal(p))
            if k == 0 or alloc - used >= k:
                out.append(name)
        return out

    def _post(self, verb: str, body: dict, http: Optional["HttpExtender"] = None):
        http = http or self.http
        assert http is not None
        return self._client.post(f"{http.url}/{verb}", body)

    def _next_http(self) -> "HttpExtender":
        """The replica this pod goes to: the primary, then each extra one in turn."""
        https = [self.http] + [h for _, h, _ in self._extra]
        self._turn = (self._turn + 1) % len(https)
        return https[self._turn]

    def schedule_one(self, pod: dict, admit: bool = True) -> ScheduleResult:
        key = pod_key(pod)
        t0 = time.perf_counter()
        http = self._next_http() if self._extra else self.http  # one replica decides the whole cycle
        cands = self._fits(pod)
        res = ScheduleResult(pod=key, node=None)
        if cands and self.use_filter:
            fr = self._post("filter", {"Pod": pod, "NodeNames": cands}, http)
            cands = fr.get("NodeNames") or []
        if not cands:
            res.error = "no feasible node"
            res.sched_ms = (time.perf_counter() - t0) * 1e3
            self.history.append(res)
            return res
        prio = self._post("sort", {"Pod": pod, "NodeNames": cands}, http)
        best = max(prio, key=lambda h: (h["Score"], -cands.index(h["Host"])))
        md = meta(pod)
        br = self._post("bind", {"PodName": md["name"], "PodNamespace": md.get("namespace", "default"), "PodUID": md.get("uid", ""),
                                 "Node": best["Host"]}, http)
        res.sched_ms = (time.perf_counter() - t0) * 1e3
        if br.get("Error"):
            res.error = br["Error"]
            self.history.append(res)
            return res
        res.node = best["Host"]
        res.score = int(best["Score"])
        res.devices = tuple(br.get("Devices") or ())
        if admit:
            t1 = time.perf_counter()
            bound = self.api.get_pod(md.get("namespace", "default"), md["name"])
            rname = self.pod_resource(bound)
            try:
                self.nodes[res.node].kubelet.admit(bound, rname)
            except AdmissionError as e:  # the kubelet rejected the pod (or its container did not start)
                res.error = f"admission: {e}"
                self.history.append(res)
                return res
            res.admit_ms = (time.perf_counter() - t1) * 1e3
            res.allocated = tuple(int(i) for i in self.nodes[res.node].kubelet.allocated[rname][key])
        self.history.append(res)
        return res

    def pending(self) -> List[dict]:
        return [p for p in self.api.list_pods() if not pod_node(p) and not pod_is_terminal(p)]

    def schedule_pending(self, admit: bool = True, concurrent: bool = False) -> List[ScheduleResult]:
        pods = sorted(self.pending(), key=lambda p: (meta(p).get("creationTimestamp", ""), int(meta(p).get("resourceVersion", 0))))
        if not concurrent:
            return [self.schedule_one(p, admit) for p in pods]
        out: Dict[str, ScheduleResult] = {}

        def go(p):
            out[pod_key(p)] = self.schedule_one(p, admit)

        ts = [threading.Thread(target=go, args=(p,)) for p in pods]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return [out[pod_key(p)] for p in pods]

    # ------------------------------------------------------------------ views
    def assignment(self, name: str, namespace: str = "default") -> Optional[PodAssignment]:
        return PodAssignment.from_annotations(obj_annotations(self.api.get_pod(namespace, name)))

    def reconcile(self) -> int:
        """One pod-resources reconciliation pass on every node (pods corrected)."""
        return sum(n.plugin.reconcile() for n in self.nodes.values())

    def used_devices(self, node: str) -> List[int]:
        assert self.extender is not None
        return sorted(self.extender.cache.refresh_node(node).used(time.time(), self.ext_cfg.assume_ttl))
