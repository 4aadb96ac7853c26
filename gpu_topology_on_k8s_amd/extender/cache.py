"""Extender node cache: topology per node + device usage rebuilt from pod annotations.

Reference: ``design.md:234`` "update the pod annotation and record the running pod on the device";
the diagram's device report carries ``isUsed``.  Here the *pod annotations are the source of truth*
(SURVEY.md §2.A A13, §5.3 (c)): usage of a node = union of ``ALIYUN_COM_GPU_GROUP`` over its
bound, non-terminal pods whose assignment is either confirmed (``ASSIGNED=true``, written by the
device plugin at Allocate) or still within the assume TTL (``ASSIGNED=false`` and
``now - ASSUME_TIME <= ttl``).  An expired assumption releases its devices (§5.3 (b)), and an
extender restart loses nothing because it rebuilds from the apiserver.

An in-memory *overlay* records binds this process made but that the apiserver view may not show yet
(watch lag / list cache), so two back-to-back binds on one node never overlap.  Pods that consume
the resource but carry no GROUP (scheduled around the extender) are counted as ``unknown`` usage:
their device ids are unknown, so only feasibility is reduced.
"""
from __future__ import annotations

import logging
import math
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional, Set, Tuple

from ..k8s.annotations import (Contract, PodAssignment, decode_node_annotations, ledger_gen, ledger_uids, parse_ledger,
                               probing_until)
from ..k8s.api import ApiError, KubeAPI
from ..k8s.objects import annotations as obj_annotations
from ..k8s.objects import labels as obj_labels
from ..k8s.objects import meta, pod_gpu_request, pod_is_terminal, pod_key, pod_node
from ..topology.model import Topology
from .ledger import LedgerStore, lease_node

log = logging.getLogger(__name__)

# a node-ledger entry whose pod no LIST has shown on the node this long after its bind is a bind that
# failed or was lost: its devices are free again (extender/scheduler.py bind).  The age is measured on
# THIS process's clock, from when this cache first saw the entry: the entry's own timestamp comes from
# the writer's clock, and an instance whose clock runs ahead of the writer's by more than the grace
# would otherwise take a bind in flight for a lapsed one.  The writer's timestamp still retires an
# entry once it is older than the grace plus LEDGER_CLOCK_SKEW_S (a ghost a restarted cache sees for
# the first time).
LEDGER_GRACE_S = 30.0
LEDGER_CLOCK_SKEW_S = 120.0

__all__ = ["Alloc", "NodeState", "ClusterCache"]


@dataclass
class Alloc:
    pod: str
    ids: Tuple[int, ...]
    assigned: bool
    assume_time: float
    source: str = "annotation"  # annotation | overlay
    cpuset: str = ""  # cores recommended to the pod at bind (<prefix>/cpuset)
    uid: str = ""  # pod UID (preemption victims are named by UID)


@dataclass
class NodeState:
    name: str
    topology: Optional[Topology] = None
    labels: Dict[str, str] = field(default_factory=dict)
    node_rv: str = ""
    node_uid: str = ""  # owner of the node's ledger Lease (garbage-collected with the node)
    allocs: Dict[str, Alloc] = field(default_factory=dict)
    unknown_pods: Dict[str, int] = field(default_factory=dict)  # pod -> devices held without a GROUP annotation
    unknown_uids: Dict[str, str] = field(default_factory=dict)  # pod UID -> pod key of unknown_pods
    capacity: int = -1  # node.status.allocatable[resource] (-1 = unknown)
    probing_until: float = 0.0  # the device plugin's re-probe mark (<prefix>/probing): skip the node until then
    # the node's allocation ledger (<prefix>/gpu-ledger, written by every extender's bind under a
    # resourceVersion precondition): pod key -> (ids, bind time).  An entry covers a bind in flight;
    # once a LIST has shown its pod on the node (`settled`) the pod's own annotation governs
    ledger: Dict[str, Tuple[Tuple[int, ...], float]] = field(default_factory=dict)
    # key -> (ids, writer time, first seen here): a re-written entry (a new incarnation of the pod name)
    # is a new entry and ages from when it was first seen
    ledger_seen: Dict[str, Tuple[Tuple[int, ...], float, float]] = field(default_factory=dict)
    # the ledger's sources (extender/ledger.py): the node's Lease and/or its Node annotation; `ledger`
    # is their union.  `lease_rv` None = no Lease for this node yet (the next bind creates it)
    ledger_lease: Dict[str, Tuple[Tuple[int, ...], float]] = field(default_factory=dict)
    ledger_node: Dict[str, Tuple[Tuple[int, ...], float]] = field(default_factory=dict)
    gen_lease: int = 0
    gen_node: int = 0
    uid_lease: Dict[str, str] = field(default_factory=dict)
    uid_node: Dict[str, str] = field(default_factory=dict)
    lease_rv: Optional[str] = None
    ledger_uid: Dict[str, str] = field(default_factory=dict)  # pod UID an entry records (extender/ledger.py)
    # ledger entries whose pod a LIST or the watch has shown bound on this node, by key -> the entry's
    # identity (bind time, pod UID).  An entry that records its pod's UID settles for good once THAT pod is seen (its own
    # annotation governs from then on, also after it ends); a re-created pod of the same name is another
    # UID and writes another entry.  An entry without a UID (a round-5 writer) is settled only while the
    # pod is shown, as before
    settled_at: Dict[str, Tuple[float, str]] = field(default_factory=dict)  # key -> (bind time, pod UID)
    # pod key -> UID of the pods the last LIST / the watch show on this node: their ledger entries
    # settle whichever arrives first (the pod's watch event or the ledger's)
    present: Dict[str, str] = field(default_factory=dict)

    @property
    def settled(self) -> Set[str]:
        return set(self.settled_at)

    def resettle(self) -> bool:
        """Recompute ``settled_at`` from ``ledger`` and ``present`` -> changed.  Call with ``lock`` held."""
        new = {}
        for k, (_, t) in self.ledger.items():
            uid = self.ledger_uid.get(k, "")
            if uid:
                if self.settled_at.get(k) == (t, uid) or self.present.get(k) == uid:
                    new[k] = (t, uid)
            elif k in self.present:
                new[k] = (t, "")
        changed = new != self.settled_at
        self.settled_at = new
        return changed
    synced_at: float = 0.0
    list_epoch: int = -1  # epoch of the newest pod LIST applied (older LISTs arriving late are stale)
    lock: threading.RLock = field(default_factory=threading.RLock, repr=False)
    # Every change of topology / labels / capacity / usage bumps `version` and clears `memo`, where the
    # extender keeps its per-pod-shape decisions for this node (sort fans out every pending pod over
    # every node; most nodes have not changed since the previous pod of the same shape).
    version: int = 0
    memo: Dict[tuple, tuple] = field(default_factory=dict, repr=False)

    def bump(self) -> None:
        """Call with ``lock`` held after any change that can alter a placement on this node."""
        self.version += 1
        self.memo.clear()

    def valid_until(self, now: float, ttl: float) -> float:
        """Time after which :meth:`used` can shrink on its own: the earliest expiry of a live
        unconfirmed assumption (``inf`` when none)."""
        t = math.inf
        for a in self.allocs.values():
            if not a.assigned and now - a.assume_time <= ttl:
                t = min(t, a.assume_time + ttl)
        g_s = min(ttl, LEDGER_GRACE_S)
        for key, (_, at) in self.ledger_live(now, ttl).items():
            t = min(t, self._first_seen(key, now) + g_s, at + g_s + LEDGER_CLOCK_SKEW_S)
        return t

    def _first_seen(self, key: str, now: float) -> float:
        seen = self.ledger_seen.get(key)
        return seen[2] if seen is not None else now

    def ledger_live_uids(self, now: float, ttl: float) -> Dict[str, str]:
        return {k: self.ledger_uid[k] for k in self.ledger_live(now, ttl) if k in self.ledger_uid}

    def ledger_live(self, now: float, ttl: float, grace: float = None) -> Dict[str, Tuple[Tuple[int, ...], float]]:
        """Ledger entries that still hold their devices: binds in flight -- seen by this cache for at
        most ``grace`` (and ``ttl``), written at most ``grace`` + LEDGER_CLOCK_SKEW_S ago by the writer's
        clock, and whose pod no LIST has shown on the node yet.  The rest are what the next ledger write
        drops (a settled pod's annotation governs; an entry past the grace is a failed bind)."""
        g_s = min(ttl, LEDGER_GRACE_S if grace is None else grace)
        return {k: (g, t) for k, (g, t) in self.ledger.items()
                if k not in self.settled_at and now - self._first_seen(k, now) <= g_s
                and now - t <= g_s + LEDGER_CLOCK_SKEW_S}

    @property
    def unknown(self) -> int:
        """Devices held by pods without a GROUP annotation (ids unknown: only feasibility shrinks)."""
        return sum(self.unknown_pods.values())

    def used(self, now: float, ttl: float) -> Set[int]:
        out: Set[int] = set()
        for a in self.allocs.values():
            if a.assigned or (now - a.assume_time) <= ttl:
                out.update(a.ids)
        for key, (ids, _) in self.ledger_live(now, ttl).items():
            if key not in self.allocs:  # being bound by another extender, not yet seen on a pod annotation
                out.update(ids)
        return out

    def free_count(self, now: float, ttl: float) -> int:
        if self.topology is None:
            return 0
        healthy = sum(1 for g in self.topology.gpus if g.healthy)
        return max(0, healthy - len(self.used(now, ttl) & {g.index for g in self.topology.gpus if g.healthy}) - self.unknown)


class ClusterCache:
    def __init__(self, api: KubeAPI, contract: Contract = Contract(), assume_ttl: float = 300.0,
                 resync_s: float = 5.0, clock: Callable[[], float] = time.time,
                 resource_aliases: Iterable[str] = (), ledger: Optional[LedgerStore] = None):
        self.api = api
        self.contract = contract
        self.ledger = ledger or LedgerStore("lease", contract=contract)
        self.ttl = float(assume_ttl)
        self.resync_s = float(resync_s)
        self.clock = clock
        self.resources = [contract.resource_name] + [r for r in resource_aliases if r != contract.resource_name]
        if contract.slice_resource and contract.slice_resource not in self.resources:
            self.resources.append(contract.slice_resource)  # time-sliced nodes' pool (topology/shares.py)
        self._nodes: Dict[str, NodeState] = {}
        self._overlay: Dict[str, Dict[str, Alloc]] = {}  # node -> pod -> alloc (binds made here)
        self._lock = threading.RLock()
        self._last_full = 0.0
        self.overlay_grace = 30.0  # seconds a bind made here may stay invisible in a lagging (cached) view
        self.consistent_lists = True  # apiserver LISTs without resourceVersion are quorum reads
        self._epoch = 0
        self._overlay_epoch: Dict[Tuple[str, str], int] = {}
        self.informer = None

    # ------------------------------------------------------------------ node objects
    def _state(self, name: str) -> NodeState:
        with self._lock:
            st = self._nodes.get(name)
            if st is None:
                st = self._nodes[name] = NodeState(name=name)
            return st

    def update_node_object(self, node: dict) -> NodeState:
        name = meta(node).get("name", "")
        st = self._state(name)
        with st.lock:
            rv = meta(node).get("resourceVersion", "")
            labels = dict(obj_labels(node))
            if st.topology is None or rv != st.node_rv or not rv or labels != st.labels:
                st.bump()
            if st.topology is None or rv != st.node_rv or not rv:
                try:
                    st.topology = decode_node_annotations(obj_annotations(node), self.contract, node_name=name)
                except Exception as e:  # malformed annotation: treat as unknown topology
                    log.warning("node %s: bad topology annotation: %s", name, e)
                    st.topology = None
                st.node_rv = rv
            st.labels = labels
            st.node_uid = str(meta(node).get("uid", "") or "")
            st.probing_until = probing_until(obj_annotations(node), self.contract)
            st.ledger_node = parse_ledger(obj_annotations(node), self.contract) if self.ledger.uses_node else {}
            st.uid_node = ledger_uids(obj_annotations(node), self.contract) if self.ledger.uses_node else {}
            st.gen_node = ledger_gen(obj_annotations(node), self.contract)
            self._apply_ledger(st)
            alloc = ((node.get("status") or {}).get("allocatable") or {})
            st.capacity = -1
            for r in self.resources:
                if r in alloc:
                    try:
                        st.capacity = int(float(alloc[r]))
                    except ValueError:
                        pass
                    break
        return st

    def _apply_ledger(self, st: NodeState) -> None:
        """With ``st.lock`` held: ``st.ledger`` = the union of the ledger's sources (the newer bind of a
        key wins), and the first-seen times of its entries (ledger_live)."""
        ledger = dict(st.ledger_node)
        uids = dict(st.uid_node)
        for k, v in st.ledger_lease.items():
            if k not in ledger or v[1] >= ledger[k][1]:
                ledger[k] = v
                uids.pop(k, None)
                if k in st.uid_lease:
                    uids[k] = st.uid_lease[k]
        changed = ledger != st.ledger or uids != st.ledger_uid
        st.ledger = ledger
        st.ledger_uid = uids
        if st.resettle() or changed:
            st.bump()
        now = self.clock()
        seen = {}
        for k, (ids, at) in ledger.items():
            prev = st.ledger_seen.get(k)
            seen[k] = prev if prev is not None and prev[:2] == (ids, at) else (ids, at, now)
        st.ledger_seen = seen

    def update_lease_object(self, node: str, lease: Optional[dict]) -> None:
        """The node's ledger Lease as read or watched (None: it does not exist / was deleted)."""
        st = self._state(node)
        with st.lock:
            if lease is None:
                st.ledger_lease, st.gen_lease, st.lease_rv, st.uid_lease = {}, 0, None, {}
            else:
                ann = obj_annotations(lease)
                st.ledger_lease = parse_ledger(ann, self.contract)
                st.uid_lease = ledger_uids(ann, self.contract)
                st.gen_lease = ledger_gen(ann, self.contract)
                st.lease_rv = str(meta(lease).get("resourceVersion", "")) or None
            self._apply_ledger(st)

    def replace_leases(self, leases: List[dict]) -> None:
        """A full LIST of the ledger namespace's Leases."""
        by_node = {}
        for lease in leases:
            n = lease_node(lease, self.contract)
            if n is not None:
                by_node[n] = lease
        with self._lock:
            names = set(self._nodes) | set(by_node)
        for n in names:
            self.update_lease_object(n, by_node.get(n))

    # ------------------------------------------------------------------ pods -> usage
    def _pod_alloc(self, pod: dict) -> Tuple[Optional[Alloc], int]:
        """(alloc, unknown_devices) of one pod already filtered to a node."""
        if pod_is_terminal(pod):
            return None, 0
        pa = PodAssignment.from_annotations(obj_annotations(pod))
        if pa is None:
            try:
                req = pod_gpu_request(pod, self.resources)
            except ValueError:
                req = 0
            return None, req
        return Alloc(pod=pod_key(pod), ids=tuple(pa.group), assigned=pa.assigned, assume_time=float(pa.assume_time),
                     cpuset=obj_annotations(pod).get(self.contract.cpuset_key, ""), uid=str(meta(pod).get("uid", ""))), 0

    def _next_epoch(self) -> int:
        with self._lock:
            self._epoch += 1
            return self._epoch

    def _rebuild(self, st: NodeState, pods: List[dict], list_epoch: int, consistent: Optional[bool] = None) -> None:
        """``list_epoch``: value of the epoch counter taken just before the pods were listed.  Called
        with ``st.lock`` held.  A LIST older than the one already applied is dropped: concurrent
        refreshes can finish out of order, and the older one may predate a bind the newer one
        already made authoritative (its overlay entry is gone).  ``consistent``: the LIST was a quorum
        read (default ``consistent_lists``); a watch-cache LIST (``resourceVersion=0``) may not show a
        bind made just before it, so its absence proves nothing."""
        consistent = self.consistent_lists if consistent is None else consistent
        if list_epoch < st.list_epoch:
            return
        st.list_epoch = list_epoch
        allocs: Dict[str, Alloc] = {}
        unknown: Dict[str, int] = {}
        unknown_uids: Dict[str, str] = {}
        seen = set()
        shown: Dict[str, str] = {}
        for p in pods:
            seen.add(pod_key(p))
            shown[pod_key(p)] = str(meta(p).get("uid", ""))
            a, u = self._pod_alloc(p)
            if u:
                unknown[pod_key(p)] = u
                unknown_uids[str(meta(p).get("uid", ""))] = pod_key(p)
            if a is not None:
                allocs[a.pod] = a
        now = self.clock()
        with self._lock:
            ov = self._overlay.get(st.name, {})
            for key in list(ov):
                a = ov[key]
                after_bind = list_epoch > self._overlay_epoch.get((st.name, key), 0)
                if key in seen:
                    if after_bind:  # a LIST started after the bind: authoritative from now on
                        del ov[key]
                    # else: this LIST shows the pod, but a LIST started before the bind may still be
                    # applied after it; keep the entry so such a stale view cannot drop the devices
                elif after_bind and consistent:
                    del ov[key]  # listed (quorum read) after the bind and absent: the pod is gone
                elif now - a.assume_time > min(self.ttl, self.overlay_grace):
                    del ov[key]  # cached/lagging lists: give up after the grace period
                else:
                    allocs[key] = a
            for key in set(self._overlay_epoch) - {(st.name, k) for k in ov}:
                if key[0] == st.name:
                    del self._overlay_epoch[key]
        if allocs != st.allocs or unknown != st.unknown_pods:  # a resync that changes nothing keeps the memo
            st.bump()
        st.allocs = allocs
        st.unknown_pods = unknown
        st.unknown_uids = unknown_uids
        # a key stays settled only while the LIST shows it: a pod name that comes back (a StatefulSet
        # pod re-created) with a new bind in flight is a new entry no LIST has shown yet
        st.present = shown
        if st.resettle():
            st.bump()
        st.synced_at = now

    def refresh_node(self, name: str) -> NodeState:
        """Authoritative re-read of one node, its ledger Lease and its pods (used before every bind).

        The pods are read last, from the apiserver's watch cache but no older than the node and Lease
        just read (``resourceVersionMatch=NotOlderThan``): an etcd range over every pod of the cluster
        per bind is not needed for the ordering that matters.  A ledger entry is dropped only by a
        write made after its writer saw the pod bound, so a pod LIST at least as new as the ledger
        shows every pod whose entry is gone.  A cache that cannot catch up (504), or an apiserver that
        refuses the parameter, gets a consistent read instead."""
        node = self.api.get_node(name)
        st = self.update_node_object(node)
        floor = _rv_int(meta(node).get("resourceVersion"))
        if self.ledger.uses_lease:
            lease = self.ledger.read_lease(self.api, name)
            self.update_lease_object(name, lease)
            if lease is not None:
                lrv = _rv_int(meta(lease).get("resourceVersion"))
                floor = None if floor is None or lrv is None else max(floor, lrv)
        epoch = self._next_epoch()
        pods = None
        if floor is not None:
            try:
                pods = self.api.list_pods(node_name=name, not_older_than=str(floor))
            except ApiError as e:
                if e.code not in (400, 422, 504):
                    raise
                log.info("pod LIST of %s not older than %s: %s; reading consistently", name, floor, e)
        if pods is None:
            pods = self.api.list_pods(node_name=name)
        with st.lock:
            self._rebuild(st, pods, epoch)
        return st

    def replace_nodes(self, nodes: List[dict]) -> None:
        """A full node LIST: update every node, forget the ones that are gone."""
        names = set()
        for node in nodes:
            names.add(self.update_node_object(node).name)
        with self._lock:
            for gone in set(self._nodes) - names:
                del self._nodes[gone]

    def replace_pods(self, pods: List[dict], epoch: Optional[int] = None, consistent: Optional[bool] = None) -> None:
        """A full pod LIST: rebuild every known node's usage from it."""
        epoch = self._next_epoch() if epoch is None else epoch
        by_node: Dict[str, List[dict]] = {}
        for p in pods:
            n = pod_node(p)
            if n:
                by_node.setdefault(n, []).append(p)
        with self._lock:
            names = set(self._nodes) | set(by_node)  # a pod LIST may land before the node LIST
        for name in names:
            st = self._state(name)
            with st.lock:
                self._rebuild(st, by_node.get(name, []), epoch, consistent)

    def sync_all(self) -> None:
        """Cluster-wide LIST of nodes + pods (polling mode, or the informer's safety resync).
        Takes node locks one at a time and never while holding one (callers must not either)."""
        epoch = self._next_epoch()
        nodes = self.api.list_nodes()
        pods = self.api.list_pods()
        self.replace_nodes(nodes)
        self.replace_pods(pods, epoch)
        with self._lock:
            self._last_full = self.clock()

    def maybe_sync(self) -> None:
        if self.informer is None and self.clock() - self._last_full >= self.resync_s:
            self.sync_all()

    # ------------------------------------------------------------------ informer (LIST+WATCH)
    def attach_informer(self, informer) -> None:
        """Drive this cache from a :class:`~..k8s.informer.Informer`: its LISTs replace the view, its
        WATCH events patch it, and :meth:`get` stops polling once it has synced."""
        self.informer = informer

    def begin_list(self, kind: str) -> Optional[int]:
        """Informer hook, called just before a LIST request: the epoch that LIST is applied under.
        Taking it after the LIST returned would let a bind that completed (:meth:`bound`) between
        the request and its arrival look older than the LIST, so the LIST — which cannot show that
        pod — would drop the bind's overlay entry and free its devices until the WATCH event."""
        return self._next_epoch() if kind == "Pod" else None

    def make_informer(self, **kw):
        """The LIST+WATCH informer that drives this cache in production (k8s/informer.py): paginated
        watch-cache LISTs, pods filtered server-side to the non-terminal ones, objects trimmed to the
        fields the cache reads, watches resumed rather than relisted.  Attached, not started."""
        from ..k8s.informer import Informer
        from ..k8s.objects import LIVE_POD_SELECTOR, trim_node, trim_pod

        prefix = self.contract.prefix

        def transform(kind: str, o: dict) -> dict:
            if kind == "Lease":
                return o
            return trim_pod(o, prefix) if kind == "Pod" else trim_node(o, prefix)

        kw.setdefault("field_selectors", {"Pod": LIVE_POD_SELECTOR})
        kw.setdefault("transform", transform)
        if self.ledger.uses_lease:  # the other extenders' binds in flight
            kw.setdefault("kinds", ("Node", "Pod", "Lease"))
            kw.setdefault("namespaces", {"Lease": self.ledger.namespace})
        inf = Informer(self.api, self.on_list, self.on_event, begin_list=self.begin_list, **kw)
        self.attach_informer(inf)
        return inf

    def on_list(self, kind: str, items: List[dict], epoch: Optional[int] = None, consistent: Optional[bool] = None) -> None:
        if kind == "Node":
            self.replace_nodes(items)
        elif kind == "Pod":
            self.replace_pods(items, epoch, consistent)
        elif kind == "Lease":
            self.replace_leases(items)
        with self._lock:
            self._last_full = self.clock()

    def informed(self) -> bool:
        return self.informer is not None and self.informer.synced

    def get(self, name: str, node_obj: Optional[dict] = None, sync: bool = True) -> NodeState:
        """Cached state of a node for scoring/filtering.

        With a synced informer this never calls the apiserver.  Otherwise a stale cache is
        refreshed with ONE cluster-wide sync (list nodes + list pods: two API calls however many
        candidates the scheduler sends), not per node.  ``sync=False`` (bind, which refreshes its
        node itself and holds the node lock) never syncs: :meth:`sync_all` takes every node's lock,
        so calling it under one can deadlock two binds on different nodes.  ``node_obj`` (scheduler
        sent full Node objects) refreshes the node's topology/labels without an API call.
        """
        stale = self.clock() - self._last_full >= self.resync_s or name not in self._nodes
        # polling mode only: with an informer attached (synced or still listing) the cluster is never
        # re-listed per request (the extender declines decisions until the informer has synced)
        if sync and stale and self.informer is None:
            try:
                self.sync_all()
            except Exception as e:
                log.warning("cache sync failed: %s", e)
        st = self.update_node_object(node_obj) if node_obj is not None else self._state(name)
        # node unknown to the last sync (e.g. just created): read it directly.  An informer's view is
        # authoritative: a node it has not delivered yet simply has no topology for now
        if sync and st.synced_at == 0.0 and self.informer is None:
            try:
                self.refresh_node(name)
            except Exception as e:
                log.warning("refresh of node %s failed: %s", name, e)
        return st

    # ------------------------------------------------------------------ writes made by this process
    def assume(self, node: str, pod: str, ids: Iterable[int], at: Optional[float] = None, cpuset: str = "",
               uid: str = "") -> None:
        a = Alloc(pod=pod, ids=tuple(int(i) for i in ids), assigned=False, assume_time=at if at is not None else self.clock(),
                  source="overlay", cpuset=cpuset, uid=uid)
        with self._lock:
            self._overlay.setdefault(node, {})[pod] = a
            # pending until :meth:`bound`: a LIST taken while the pod is still unbound does not show
            # it on the node and must not drop the assumption (the refresh before a concurrent bind
            # on the same node runs outside the node lock)
            self._overlay_epoch[(node, pod)] = math.inf
        st = self._state(node)
        with st.lock:
            st.allocs[pod] = a
            st.bump()

    def bound(self, node: str, pod: str) -> None:
        """The binding of an assumed pod was accepted: a LIST started after this point must show the
        pod on the node, so one that does not proves the pod is gone."""
        with self._lock:
            if (node, pod) in self._overlay_epoch:
                self._overlay_epoch[(node, pod)] = self._next_epoch()

    def forget(self, node: str, pod: str) -> None:
        with self._lock:
            self._overlay.get(node, {}).pop(pod, None)
        st = self._state(node)
        with st.lock:
            st.allocs.pop(pod, None)
            st.bump()

    # ------------------------------------------------------------------ watch events (fake / informer)
    def on_event(self, event: str, kind: str, obj: dict) -> None:
        if kind == "Lease":
            n = lease_node(obj, self.contract)
            if n is not None:
                self.update_lease_object(n, None if event == "DELETED" else obj)
            return
        if kind == "Node":
            if event == "DELETED":
                with self._lock:
                    self._nodes.pop(meta(obj).get("name", ""), None)
            else:
                self.update_node_object(obj)
            return
        if kind != "Pod":
            return
        node = pod_node(obj)
        if not node:
            return
        st = self._state(node)
        key = pod_key(obj)
        with st.lock:
            st.bump()
            if event == "DELETED" or pod_is_terminal(obj):
                st.allocs.pop(key, None)
                st.unknown_pods.pop(key, None)
                st.present.pop(key, None)  # its ledger entry stays settled: the pod was seen, then ended
                with self._lock:
                    self._overlay.get(node, {}).pop(key, None)
                return
            # the watch shows the pod bound on the node, as a LIST would: from now on its own annotation
            # governs, and its ledger entry no longer holds devices once the pod ends
            st.present[key] = str(meta(obj).get("uid", ""))
            st.resettle()
            a, u = self._pod_alloc(obj)
            if a is not None:
                st.allocs[key] = a  # the apiserver has the assignment: authoritative over the overlay
                st.unknown_pods.pop(key, None)
                with self._lock:
                    self._overlay.get(node, {}).pop(key, None)
            else:
                if u:
                    st.unknown_pods[key] = u
                    st.unknown_uids[str(meta(obj).get("uid", ""))] = key
                else:
                    st.unknown_pods.pop(key, None)
                if key in st.allocs and st.allocs[key].source == "annotation":
                    del st.allocs[key]  # GROUP removed (bind rollback)

    def nodes(self) -> List[NodeState]:
        with self._lock:
            return list(self._nodes.values())

    def snapshot(self) -> Dict[str, dict]:
        now = self.clock()
        out = {}
        for st in self.nodes():
            with st.lock:
                out[st.name] = {
                    "devices": st.topology.n if st.topology else 0,
                    "used": sorted(st.used(now, self.ttl)),
                    "unknown": st.unknown,
                    "free": st.free_count(now, self.ttl),
                    "allocs": {k: {"ids": list(a.ids), "assigned": a.assigned, "assume_time": a.assume_time, "source": a.source,
                                   "cpuset": a.cpuset}
                               for k, a in st.allocs.items()},
                    "labels": st.labels,
                }
        return out


def _rv_int(rv) -> Optional[int]:
    """A resourceVersion as the etcd revision it is, or None (opaque to this client: no floor)."""
    try:
        return int(str(rv))
    except (TypeError, ValueError):
        return None
