"""Topology-aware scheduler-extender core: filter, prioritize ("sort") and bind.

Reference (``design.md:88-234``):
  * Policy registers one extender with ``PrioritizeVerb: sort`` and ``bindVerb: bind`` and no filter
    (``design.md:92-117``: count feasibility is left to the default scheduler).
  * prioritize: per candidate node, find the best free-GPU combination for the request and return
    its affinity score (``design.md:118,123-129``), 0..10.
  * bind: recompute the best combination on the chosen node, write ``ALIYUN_COM_GPU_GROUP``,
    ``ALIYUN_COM_GPU_ASSIGNED=false``, ``ALIYUN_COM_GPU_ASSUME_TIME=<now>`` and bind
    (``design.md:119,223-232``).

This implementation adds:
  * an optional filter verb that rejects nodes with no topology, too few free devices, or the wrong
    GPU model (heterogeneous-cluster quota, Gaia B7);
  * node scores normalised over the candidate set: the best feasible node gets 10 and every other
    loses one point per ``score_resolution`` of relative objective gap, so a measured degraded link
    (a fraction of a percent of an 8-GPU set's mean cost) still decides between nodes;
  * CPU affinity (``design.md:135-147`` tie-break, Gaia B6): a degraded PCIe host link, a slow HBM
    stack and the SLIT distance from the pod's preferred NUMA node raise a device's access cost, and
    bind writes the chosen devices' core slices (``<prefix>/cpuset``) and NUMA nodes on the pod;
  * fractional requests (Gaia Fragment, Alg. 2) as XCP partitions of ONE physical GPU on
    CPX/DPX/QPX nodes, or as time slices of one GPU on a node whose device plugin runs with
    ``--time-slices`` (topology/shares.py), selected by the ``<prefix>/gpu-fraction`` pod annotation;
    time slices are their own resource pool (``Contract.slice_resource``, default
    ``amd.com/gpu-slice``): ``amd.com/gpu`` means a whole GPU on every node (Gaia's heterogeneous
    quota against resource-pool pollution, paper p.3 §III.A), and the filter names every mismatch;
  * per-node locking + an assume overlay so concurrent binds never overlap (BASELINE config 4);
  * three selectable policies: ``exact`` (default, :func:`placement.select`), ``gaia`` (cost-tree
    Alg. 1-4) and ``design`` (the reference's greedy/Prim, for parity experiments);
  * k8s Events on bind success / failure, and binds refused for pods this extender does not manage.
"""
from __future__ import annotations

import dataclasses
import logging
import math
import random
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

from ..k8s.annotations import ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GROUP, Contract, PodAssignment
from ..k8s.api import ApiError, Conflict, KubeAPI
from ..k8s.events import record_event
from ..k8s.objects import annotations as obj_annotations
from ..k8s.objects import labels as obj_labels
from ..k8s.objects import meta, pod_device_steps, pod_gpu_request, pod_key
from ..placement import NoFeasiblePlacement, PlacementPolicy, place_fraction, select
from ..placement.core import node_packing_term, select_with
from ..placement.numa_align import plan as numa_plan
from ..placement.numa_align import tm_from_labels
from ..placement.gaia import gaia_schedule, tree_from_topology
from ..placement.legacy import design_greedy_select
from ..topology.cpus import access_costs, recommended_cpuset
from ..topology.model import Topology
from ..topology.shares import slices_per_gpu
from .cache import LEDGER_GRACE_S, ClusterCache, NodeState
from .ledger import LedgerStore
from .metrics import ExtenderMetrics

log = logging.getLogger(__name__)

__all__ = ["ExtenderConfig", "TopologyExtender", "Decision", "MalformedPod", "normalized_scores"]


class MalformedPod(ValueError):
    """The pod's GPU request cannot be read (a quantity that is not a non-negative integer, a
    container that is not an object): the verbs answer without scoring or binding it."""

MAX_EXTENDER_PRIORITY = 10  # k8s.io/kube-scheduler/extender/v1 MaxExtenderPriority


@dataclass
class ExtenderConfig:
    contract: Contract = field(default_factory=Contract)
    resource_aliases: Tuple[str, ...] = ("aliyun.com/gpu", "aliyun.com/gpu-count")
    policy_name: str = "exact"  # exact | gaia | design
    policy: PlacementPolicy = field(default_factory=PlacementPolicy)
    assume_ttl: float = 300.0
    resync_s: float = 5.0
    require_model_match: bool = True
    bind_retries: int = 3
    seed: Optional[int] = None
    decision_cache: int = 4096  # LRU entries; 0 disables (random tie-breaks are never cached)
    # relative objective gap worth one score point below the best candidate (prioritize)
    score_resolution: float = 0.005
    cpu_affinity: bool = True  # access term from the devices' local cores (A16 / Gaia B6)
    # pods whose spec.schedulerName is not listed are refused at bind (empty = any scheduler)
    scheduler_names: Tuple[str, ...] = ()
    events: bool = True
    # the node allocation ledger (Contract.ledger_key): every bind records its device set on the Node
    # with a resourceVersion precondition, so concurrent extender instances cannot overlap; a 409
    # re-reads the node and re-decides, up to `ledger_attempts` times
    ledger: bool = True
    ledger_attempts: int = 8
    # where the ledger lives (extender/ledger.py): one coordination.k8s.io Lease per node in
    # `ledger_namespace` ("lease"), the round-5 Node annotation ("node"), or both during a rolling
    # upgrade between the two ("both"; docs/MIGRATION.md)
    ledger_store: str = "lease"
    ledger_namespace: str = "kube-system"
    # a bind holds its node's lock while it refreshes, decides, records and binds, and the informer's
    # events for that node wait on it: the ledger retry loop gives up after this long
    bind_budget_s: float = 10.0


@dataclass
class Decision:
    node: str
    ids: Tuple[int, ...]
    score: float
    objective: float
    policy: str
    micros: float
    cpuset: str = ""
    rank: float = float("nan")  # objective + node-level packing term: what nodes are compared by


class _held:
    """Context manager observing how long a block ran (a lock held) into a Histogram."""

    def __init__(self, hist):
        self.hist = hist

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.hist.observe(time.perf_counter() - self.t0)
        return False


def normalized_scores(objectives: Dict[str, float], resolution: float = 0.005) -> Dict[str, int]:
    """Node scores for one pod: 10 for the lowest objective, one point less per ``resolution`` of
    relative gap (rounded up, so any strictly worse node scores strictly lower), never below 1 (a
    feasible node always beats an infeasible one, which scores 0)."""
    if not objectives:
        return {}
    best = min(objectives.values())
    out = {}
    for n, j in objectives.items():
        gap = (j - best) / max(abs(best), 1e-12)
        pts = 0 if gap <= 1e-9 else math.ceil(gap / resolution - 1e-9)
        out[n] = int(max(1, MAX_EXTENDER_PRIORITY - pts))
    return out


class TopologyExtender:
    def __init__(self, api: KubeAPI, config: Optional[ExtenderConfig] = None, metrics: Optional[ExtenderMetrics] = None,
                 clock=time.time):
        self.api = api
        self.cfg = config or ExtenderConfig()
        self.clock = clock
        self.ledger = LedgerStore(self.cfg.ledger_store, self.cfg.ledger_namespace, self.cfg.contract)
        self.cache = ClusterCache(api, self.cfg.contract, self.cfg.assume_ttl, self.cfg.resync_s, clock=clock,
                                  resource_aliases=self.cfg.resource_aliases, ledger=self.ledger)
        self.metrics = metrics or ExtenderMetrics()
        self.metrics.attach_cache(self.cache, self.cfg.assume_ttl, clock)
        self._rng = random.Random(self.cfg.seed)
        self._bind_lock = threading.Lock()
        # Placement decisions are a pure function of (node topology object, used set, healthy set,
        # access costs, k, fraction) under a deterministic policy: kube-scheduler asks sort for every
        # pending pod x candidate node, and on a large cluster most nodes have not changed since the
        # last pod of the same size.
        self._cache: "OrderedDict[tuple, Tuple[Tuple[int, ...], float, float, Topology]]" = OrderedDict()
        self._cache_lock = threading.Lock()

    # ------------------------------------------------------------------ helpers
    @property
    def resources(self) -> List[str]:
        return self.cache.resources

    def request_of(self, pod: Dict[str, Any]) -> int:
        """Devices the pod asks for; a quantity that is not a non-negative integer raises
        :class:`MalformedPod` (the verbs answer it without scoring or binding the pod)."""
        try:
            return pod_gpu_request(pod, self.resources)
        except ValueError as e:
            raise MalformedPod(f"malformed GPU request: {e}") from None

    def fraction_of(self, pod: Dict[str, Any]) -> Optional[float]:
        """``<prefix>/gpu-fraction`` (0 < m < 1) or None; malformed values raise ValueError."""
        raw = obj_annotations(pod).get(self.cfg.contract.fraction_key)
        if raw is None or str(raw).strip() == "":
            return None
        m = float(raw)
        if not 0.0 < m < 1.0:
            raise ValueError(f"{self.cfg.contract.fraction_key} must be in (0, 1), got {raw!r}")
        return m

    def memory_of(self, pod: Dict[str, Any]) -> Optional[int]:
        """``<prefix>/gpu-memory`` in bytes ("96Gi", "100G", "1e11") or None; malformed values raise ValueError."""
        raw = obj_annotations(pod).get(self.cfg.contract.memory_key)
        if raw is None or str(raw).strip() == "":
            return None
        txt = str(raw).strip()
        units = {"Ki": 2**10, "Mi": 2**20, "Gi": 2**30, "Ti": 2**40, "K": 10**3, "M": 10**6, "G": 10**9, "T": 10**12}
        mult = 1
        for u in sorted(units, key=len, reverse=True):
            if txt.endswith(u):
                txt, mult = txt[: -len(u)], units[u]
                break
        v = float(txt) * mult
        if not (v == v and v != float("inf")):  # nan / inf: no HBM share can be sized from it
            raise ValueError(f"{self.cfg.contract.memory_key} must be a finite size, got {raw!r}")
        b = int(v)
        if b <= 0:
            raise ValueError(f"{self.cfg.contract.memory_key} must be positive, got {raw!r}")
        return b

    def numa_preference(self, pod: Dict[str, Any]) -> Optional[List[int]]:
        """NUMA node(s) the pod's host threads run on (``<prefix>/numa-preference: "1"``), if stated."""
        raw = obj_annotations(pod).get(self.cfg.contract.numa_pref_key)
        if not raw:
            return None
        try:
            return [int(x) for x in str(raw).split(",") if x.strip()]
        except ValueError:
            return None

    def _model_ok(self, want: Optional[str], st: NodeState) -> Tuple[bool, str]:
        """Heterogeneous-cluster quota (Gaia B7): a pod never receives a mix of GPU models, and a
        pod asking for a model (``want``: its annotation or label) only lands on nodes advertising it."""
        t = st.topology
        models = {g.model for g in t.gpus} if t is not None else set()
        node_model = st.labels.get(self.cfg.contract.label_model)
        if len(models) > 1:
            return False, f"node mixes GPU models {sorted(models)}"
        if want and self.cfg.require_model_match:
            have = node_model or (next(iter(models)) if models else "")
            if have != want:
                return False, f"pod wants GPU model {want}, node has {have or 'unknown'}"
        return True, ""

    def _cacheable(self) -> bool:
        return self.cfg.decision_cache > 0 and self.cfg.policy.tie_break != "random"

    def _choose_cached(self, t: Topology, used: Sequence[int], k: int, access=None,
                       fraction: Optional[float] = None, multi: bool = False) -> Tuple[Tuple[int, ...], float, float]:
        if not self._cacheable():
            return self._choose(t, used, k, access, fraction, multi)
        # the Topology object is replaced whenever the node annotation changes (new resourceVersion)
        acc_key = None if access is None else tuple(round(float(x), 9) for x in access)
        key = (id(t), tuple(used), tuple(g.healthy for g in t.gpus), k, self.cfg.policy_name, acc_key, fraction, multi)
        with self._cache_lock:
            hit = self._cache.get(key)
            if hit is not None and hit[3] is t:
                self._cache.move_to_end(key)
                self.metrics.cache(True)
                return hit[:3]
        res = self._choose(t, used, k, access, fraction, multi)  # NoFeasiblePlacement propagates uncached
        with self._cache_lock:
            self._cache[key] = res + (t,)  # keeps t alive, so id(t) cannot be reused while cached
            while len(self._cache) > self.cfg.decision_cache:
                self._cache.popitem(last=False)
        self.metrics.cache(False)
        return res

    def _choose(self, t: Topology, used: Sequence[int], k: int, access=None,
                fraction: Optional[float] = None, multi: bool = False) -> Tuple[Tuple[int, ...], float, float]:
        """(ids, absolute score 0..10, objective) under the configured policy; raises NoFeasiblePlacement."""
        from ..placement.core import Problem, evaluate, score_from_objective

        name = self.cfg.policy_name
        if fraction is not None:
            ids = place_fraction(t, k, used, access)
            name = "fragment"
        elif name == "exact":
            pl = select(t, k, used=used, policy=self.cfg.policy, rng=self._rng, access=access, nic_aware=multi)
            return pl.ids, pl.score, pl.objective
        elif name == "gaia":
            tree = tree_from_topology(t, used=[u for u in used])
            for g in t.gpus:
                if not g.healthy and g.index not in used:
                    tree.mark_used([g.index])
            ids = gaia_schedule(tree, k, tie_break=self.cfg.policy.tie_break, rng=self._rng)
        elif name == "design":
            unhealthy = [g.index for g in t.gpus if not g.healthy]
            ids = design_greedy_select(t.cost, list(used) + unhealthy, k)
        else:
            raise ValueError(f"unknown policy {name!r}")
        if len(ids) != k:
            raise NoFeasiblePlacement(f"{name}: no {k}-device placement")
        j, _ = evaluate(Problem.from_topology(t, used, access, partition_aware=self.cfg.policy.partition_aware, nic_aware=multi),
                        ids, self.cfg.policy)
        return tuple(sorted(int(i) for i in ids)), score_from_objective(j), j

    def _choose_aligned(self, t: Topology, used: Sequence[int], k: int, access, multi: bool,
                        steps: Sequence[Tuple[int, str]], tm) -> Tuple[Optional[Tuple[int, ...]], str]:
        """The GROUP on a node whose kubelet runs the Topology Manager: the devices the kubelet will
        offer container by container (placement/numa_align.py), the placement core choosing wherever
        the kubelet leaves the choice to the plugin.  (None, why) when the kubelet would reject the pod."""
        def choose(n: int, offered: Sequence[int], must: Sequence[int]) -> Sequence[int]:
            if must:
                return select_with(t, n, offered, must, self.cfg.policy)
            return select(t, n, used=[i for i in range(t.n) if i not in set(offered)], policy=self.cfg.policy,
                          rng=self._rng, access=access, nic_aware=multi).ids

        ids, why = numa_plan(t, used, steps, tm, choose)
        if ids is not None and len(ids) != k:
            return None, f"the kubelet's topology manager would allocate {len(ids)} devices, the pod requests {k}"
        return ids, why

    def _rate(self, t: Topology, used: Sequence[int], ids: Sequence[int], access, multi: bool) -> Tuple[float, float]:
        from ..placement.core import Problem, evaluate, score_from_objective

        j, _ = evaluate(Problem.from_topology(t, used, access, partition_aware=self.cfg.policy.partition_aware, nic_aware=multi),
                        list(ids), self.cfg.policy)
        return score_from_objective(j), j

    def request_unit(self, pod: Dict[str, Any]) -> Tuple[Optional[str], str]:
        """Which pool the pod draws from: ``"gpu"`` (whole GPUs: the resource name and its aliases) or
        ``"slice"`` (``Contract.slice_resource``, time slices of sliced nodes); (None, reason) when it
        asks for both — the two pools are never mixed in one pod."""
        sl = self.cfg.contract.slice_resource
        whole = pod_gpu_request(pod, [r for r in self.resources if r != sl])
        slices = pod_gpu_request(pod, [sl]) if sl else 0
        if whole and slices:
            return None, f"pod requests both whole GPUs and {sl}: use one pool"
        return ("slice" if slices else "gpu"), ""

    def _pod_shape(self, pod: Dict[str, Any], k: int) -> Tuple[Optional[tuple], str]:
        """What a placement depends on from the pod: (k, fraction, NUMA preference, GPU model,
        multi-node, memory, pool unit, device steps), parsed once per request; (None, reason) for a
        malformed one.  The steps (``(count, kind)`` per container, kubelet admission order) matter
        on nodes with a Topology Manager, which aligns each container on its own."""
        try:
            fraction = self.fraction_of(pod)
            mem = self.memory_of(pod)
            unit, why = self.request_unit(pod)
            steps = tuple((n, kind) for _, n, kind in pod_device_steps(pod, self.resources))
        except ValueError as e:
            return None, str(e)
        if unit is None:
            return None, why
        if mem is not None and fraction is None:
            fraction = 0.0  # a memory-sized share of one GPU: the Fragment path, sized by HBM below
        numa = self.numa_preference(pod)
        want = obj_annotations(pod).get(self.cfg.contract.pod_model_key) or obj_labels(pod).get(self.cfg.contract.pod_model_key)
        return (k, fraction, tuple(numa) if numa else None, want, self.multi_node(pod), mem, unit, steps), ""

    def multi_node(self, pod: Dict[str, Any]) -> bool:
        """A member of a multi-node job: ``<prefix>/multi-node: "true"``, or it requests an RDMA
        resource (any resource name containing ``rdma``)."""
        if str(obj_annotations(pod).get(self.cfg.contract.multi_node_key, "")).strip().lower() in ("1", "true", "yes"):
            return True
        spec = pod.get("spec")
        cs = spec.get("containers") if isinstance(spec, dict) else None
        for c in cs if isinstance(cs, list) else []:
            res = c.get("resources") if isinstance(c, dict) else None
            for part in ("limits", "requests"):
                vals = res.get(part) if isinstance(res, dict) else None
                if isinstance(vals, dict) and any("rdma" in str(name).lower() for name in vals):
                    return True
        return False

    def _eval_state(self, pod: Dict[str, Any], name: str, st: NodeState, k: int,
                    shape: Optional[tuple] = None) -> Tuple[Optional[Decision], str]:
        """Decision for ``pod`` on the node state ``st`` as cached now.  Never calls the apiserver,
        so it may run under the node lock (bind).  Memoised per node on the pod's shape (k, fraction,
        NUMA preference, GPU model) until the node state changes or a live assumption expires."""
        if shape is None:
            shape, why = self._pod_shape(pod, k)
            if shape is None:
                return None, why
        _, fraction, numa, want, multi, mem, unit, steps = shape
        with st.lock:
            now = self.clock()
            if st.probing_until > now:
                # the device plugin is re-measuring the node's links (deviceplugin/plugin.py reprobe):
                # a pod placed now would share them with the probe; not memoised (the mark expires)
                self.metrics.probing_skips.inc()
                return None, f"link probe in progress on this node (until {int(st.probing_until)})"
            if self._cacheable():
                hit = st.memo.get(shape)
                if hit is not None and hit[0] <= now <= hit[1]:
                    self.metrics.cache(True)
                    return hit[2], hit[3]
            d, why = self._eval_state_uncached(st, name, k, fraction, numa, want, now, multi, mem, unit, steps)
            if self._cacheable():
                st.memo[shape] = (now, st.valid_until(now, self.cfg.assume_ttl), d, why)
            return d, why

    def _pool_ok(self, t: Topology, unit: str) -> Tuple[bool, str]:
        """Resource pools stay apart (Gaia paper p.3 §III.A, resource pool pollution): a time-sliced
        node serves only slice requests, every other node only whole-device requests."""
        c = self.cfg.contract
        s = slices_per_gpu(t)
        if s > 1 and unit != "slice":
            return False, (f"node shares its GPUs as {c.slice_resource} ({s} per GPU); {c.resource_name} requests "
                           f"whole GPUs, which this node does not offer")
        if s <= 1 and unit == "slice":
            return False, (f"node has no time slices ({c.slice_resource} is offered by nodes labelled "
                           f"{c.time_slices_label}=S)")
        return True, ""

    def _eval_state_uncached(self, st: NodeState, name: str, k: int, fraction: Optional[float], numa, want,
                             now: float, multi: bool = False, mem: Optional[int] = None,
                             unit: str = "gpu", steps: Sequence[Tuple[int, str]] = ()) -> Tuple[Optional[Decision], str]:
        t = st.topology
        if t is None:
            return None, "node has no GPU topology annotation"
        ok, why = self._model_ok(want, st)
        if not ok:
            return None, why
        ok, why = self._pool_ok(t, unit)
        if not ok:
            return None, why
        if fraction is not None:
            sizes = {}
            for g in t.gpus:
                sizes[g.physical] = sizes.get(g.physical, 0) + 1
            per_gpu = max(sizes.values()) if sizes else 1
            if per_gpu <= 1 and mem is not None and fraction == 0.0:
                # whole GPUs: a memory size only has to fit one device, then it is an ordinary request
                if any(0 < g.vram_bytes < mem for g in t.gpus):
                    return None, f"gpu-memory {mem} B exceeds a device on this node"
                fraction = None
            elif per_gpu <= 1:
                return None, "fractional GPU requests need a partitioned (CPX/DPX/QPX) or time-sliced node"
        if fraction is not None:
            need = max(1, math.ceil(fraction * per_gpu - 1e-9))
            what = f"gpu-fraction {fraction}"
            if mem is not None:
                dev_mem = min((g.vram_bytes for g in t.gpus if g.vram_bytes > 0), default=0)
                if dev_mem <= 0:
                    return None, "node does not publish device memory sizes: gpu-memory cannot be sized"
                need_mem = math.ceil(mem / dev_mem - 1e-9)
                if need_mem > per_gpu:
                    return None, f"gpu-memory {mem} B exceeds one GPU on this node ({per_gpu} x {dev_mem} B)"
                if need_mem > need:
                    need, what = need_mem, f"gpu-memory {mem} B ({dev_mem} B per device)"
            if need != k:
                return None, (f"{what} is {need} of {per_gpu} partitions per GPU on this node, "
                              f"but the pod requests {k} devices")
        used = sorted(st.used(now, self.cfg.assume_ttl))
        free = st.free_count(now, self.cfg.assume_ttl)
        if free < k:
            return None, f"insufficient free devices: need {k}, free {free}"
        access = access_costs(t, numa) if self.cfg.cpu_affinity else None
        t0 = time.perf_counter()
        tm = tm_from_labels(st.labels, self.cfg.contract.prefix)
        try:
            if tm.active and fraction is None and steps:
                ids, why = self._choose_aligned(t, used, k, access, multi, steps, tm)
                if ids is None:
                    return None, why
                score, obj = self._rate(t, used, ids, access, multi)
            else:
                ids, score, obj = self._choose_cached(t, used, k, access, fraction, multi)
        except NoFeasiblePlacement as e:
            return None, str(e)
        us = (time.perf_counter() - t0) * 1e6
        rank = obj + node_packing_term(free, k, t.n, self.cfg.policy)
        return Decision(node=name, ids=ids, score=score, objective=obj,
                        policy="fragment" if fraction is not None else self.cfg.policy_name, micros=us, rank=rank), ""

    def _node_eval(self, pod: Dict[str, Any], name: str, node_obj: Optional[dict], k: int,
                   shape: Optional[tuple] = None) -> Tuple[Optional[Decision], str]:
        st = self.cache.get(name, node_obj)  # may sync the cache: never call with a node lock held
        return self._eval_state(pod, name, st, k, shape)

    # ------------------------------------------------------------------ verbs
    NOT_READY = "gpu-topology extender is still listing the cluster (informer not synced); retry"

    @property
    def ready(self) -> bool:
        """Decisions can be made: polling mode, or the informer has listed every kind once.  Until
        then filter and sort decline GPU pods (kube-scheduler retries them) instead of deciding on an
        empty view, and nothing falls back to cluster-wide LISTs (at 100,000 pods one takes ~50 s and
        GBs).  Bind needs no gate: it decides on its own refresh of the node (its object, its pods, its
        ledger Lease) under the node lock."""
        return self.cache.informer is None or self.cache.informed()

    def filter(self, pod: Dict[str, Any], node_names: Sequence[str], node_objs: Optional[Dict[str, dict]] = None):
        """-> (passing node names, {failed node: reason})."""
        t0 = time.perf_counter()
        try:
            k = self.request_of(pod)
        except MalformedPod as e:
            return [], {n: str(e) for n in node_names}
        if k and not self.ready:
            self.metrics.request("filter", "not_ready")
            return [], {n: self.NOT_READY for n in node_names}
        ok: List[str] = []
        failed: Dict[str, str] = {}
        shape, bad = self._pod_shape(pod, k) if k else (None, "")
        for n in node_names:
            if k == 0:
                ok.append(n)
                continue
            if shape is None:
                failed[n] = bad
                continue
            d, why = self._node_eval(pod, n, (node_objs or {}).get(n), k, shape)
            if d is None:
                failed[n] = why
            else:
                ok.append(n)
        self.metrics.observe("filter", time.perf_counter() - t0)
        return ok, failed

    def prioritize(self, pod: Dict[str, Any], node_names: Sequence[str], node_objs: Optional[Dict[str, dict]] = None):
        """-> [(host, score 0..10)]: infeasible nodes 0 (the reference has no filter verb), feasible
        nodes :func:`normalized_scores` of their best placement's objective."""
        t0 = time.perf_counter()
        try:
            k = self.request_of(pod)
        except MalformedPod:
            return [(n, 0) for n in node_names]
        if k and not self.ready:
            self.metrics.request("prioritize", "not_ready")
            return [(n, 0) for n in node_names]
        objs: Dict[str, float] = {}
        shape, _ = self._pod_shape(pod, k) if k else (None, "")
        for n in node_names:
            if shape is None:
                continue
            d, _ = self._node_eval(pod, n, (node_objs or {}).get(n), k, shape)
            if d is not None:
                objs[n] = d.rank if d.rank == d.rank else d.objective
                self.metrics.score(d.score)
        norm = normalized_scores(objs, self.cfg.score_resolution)
        out = [(n, norm.get(n, 0)) for n in node_names]
        self.metrics.observe("prioritize", time.perf_counter() - t0)
        return out

    def bind(self, namespace: str, name: str, uid: str, node: str) -> Optional[Decision]:
        """Choose the device set on ``node``, annotate the pod, bind it.  Raises on failure."""
        t0 = time.perf_counter()
        pod: Optional[Dict[str, Any]] = None
        try:
            pod = self.api.get_pod(namespace, name)
            k = self.request_of(pod)
            bound_to = (pod.get("spec") or {}).get("nodeName") or ""
            if bound_to:
                # a retried bind (scheduler timeout) must not rewrite a live assignment
                pa = PodAssignment.from_annotations(obj_annotations(pod))
                if bound_to == node and (k == 0 or (pa is not None and len(pa.group) == k)):
                    ids = tuple(pa.group) if pa is not None else ()
                    return Decision(node=node, ids=ids, score=float("nan"), objective=float("nan"), policy="already-bound",
                                    micros=0.0) if ids else None
                raise ApiError(409, f"pod {namespace}/{name} is already bound to {bound_to}")
            if k == 0:
                # kube-scheduler only delegates binding of pods that request a managed resource; any
                # other bind request did not come from it and is refused
                raise ApiError(400, f"pod {namespace}/{name} requests none of {self.resources}: not managed by this extender")
            sched = (pod.get("spec") or {}).get("schedulerName") or "default-scheduler"
            if self.cfg.scheduler_names and sched not in self.cfg.scheduler_names:
                raise ApiError(403, f"pod {namespace}/{name} uses scheduler {sched!r}, not one of {list(self.cfg.scheduler_names)}")
            key = pod_key(pod)
            started = time.monotonic()
            for attempt in range(max(1, self.cfg.ledger_attempts)):
                if attempt and time.monotonic() - started > self.cfg.bind_budget_s:
                    self.metrics.bind_aborts.labels("budget").inc()
                    raise ApiError(409, f"bind {namespace}/{name} on {node}: {attempt} ledger conflicts in "
                                        f"{time.monotonic() - started:.1f}s (budget {self.cfg.bind_budget_s:.0f}s)")
                st = self.cache.get(node, sync=False)
                # serialise refresh+select+annotate+bind per node (in this process).  The refresh (2 API
                # calls) runs under this node's lock, and takes no other node's: the decision must see
                # the node object and the pod LIST of ONE refresh.  Refreshed outside the lock, a
                # concurrent refresh could apply a newer node object -- whose ledger has already dropped
                # a pod its writer saw bound -- over an older LIST that does not show that pod yet; the
                # pod's devices then look free and the resourceVersion precondition (the newer object's)
                # passes: one device, two pods.
                with st.lock, _held(self.metrics.bind_lock_seconds):
                    if self.cache.refresh_node(node) is not st:
                        continue  # the node was dropped and re-created meanwhile: decide on the new state
                    d, why = self._eval_state(pod, node, st, k)
                    if d is None:
                        raise NoFeasiblePlacement(f"bind {namespace}/{name} on {node}: {why}")
                    d = dataclasses.replace(d, cpuset=recommended_cpuset(st.topology, d.ids))  # memo entries stay unshared
                    now = self.clock()
                    if self.cfg.ledger:
                        # across processes: record the set in the node's ledger, conditional on the
                        # ledger being exactly what this decision saw; another extender's bind in
                        # between -> 409
                        entries = st.ledger_live(now, self.cfg.assume_ttl)
                        entries[key] = (tuple(d.ids), now)
                        uids = st.ledger_live_uids(now, self.cfg.assume_ttl)
                        uids[key] = uid or str(meta(pod).get("uid", ""))
                        try:
                            self.ledger.write(self.api, node, entries, st.lease_rv, st.gen_lease, st.node_rv, st.gen_node,
                                              uids, node_uid=st.node_uid)
                        except Conflict:
                            self.metrics.ledger_conflicts += 1
                            self.metrics.ledger_conflict.inc()
                            log.info("bind %s on %s: ledger changed since the decision (attempt %d); re-deciding",
                                     key, node, attempt + 1)
                            continue
                        except ApiError as e:
                            if e.code == 403:  # RBAC without the ledger's verbs: say what to fix, then fail the bind
                                need = []
                                if self.ledger.uses_lease:
                                    need.append(f"`create`/`patch` on leases.coordination.k8s.io in {self.ledger.namespace}")
                                if self.ledger.uses_node:
                                    need.append("`patch` on nodes")
                                raise ApiError(403, f"bind {key} on {node}: the allocation ledger needs {' and '.join(need)} "
                                                    f"for the extender's service account (or run with --bind-ledger off "
                                                    f"for a single extender): {e}") from e
                            raise
                    return self._commit(pod, namespace, name, uid, node, key, d, st, now, time.monotonic())
            raise ApiError(409, f"bind {namespace}/{name} on {node}: the node's allocation ledger kept changing "
                                f"({self.cfg.ledger_attempts} attempts)")
        except Exception as e:
            if self.cfg.events and pod is not None:
                record_event(self.api, pod, "FailedGPUTopologyBind", f"bind to {node} failed: {e}", "Warning",
                             component="gpu-topology-extender")
            raise
        finally:
            self.metrics.observe("bind", time.perf_counter() - t0)

    def _commit(self, pod, namespace: str, name: str, uid: str, node: str, key: str, d: Decision, st: NodeState,
                now: float, recorded: Optional[float] = None) -> Decision:
        """Under ``st.lock``, the devices recorded: annotate the pod, bind it; undo everything on failure.

        ``recorded``: when the ledger entry was written (monotonic).  Another extender counts the entry
        for LEDGER_GRACE_S from when it first sees it, never before it was written; a bind that has not
        reached the apiserver's binding call within half of that (a throttled or retrying apiserver) is
        given up and rolled back rather than completed after the entry may have lapsed and the devices
        been handed out again."""
        pa = PodAssignment.assumed(d.ids, now)
        ann = pa.to_annotations()
        t = st.topology
        numa = sorted({t.gpus[i].numa for i in d.ids}) if t is not None else []
        ann[self.cfg.contract.numa_key] = ",".join(str(x) for x in numa)
        if d.cpuset:
            ann[self.cfg.contract.cpuset_key] = d.cpuset
        ann[self.cfg.contract.score_key] = f"{d.score:.3f}"
        self.cache.assume(node, key, d.ids, now, cpuset=d.cpuset, uid=uid or str(meta(pod).get("uid", "")))
        try:
            self._patch_with_retry(namespace, name, ann)
            if self.cfg.ledger and recorded is not None and time.monotonic() - recorded > LEDGER_GRACE_S / 2:
                self.metrics.bind_aborts.labels("ledger_grace").inc()
                raise ApiError(503, f"bind {key} on {node}: {time.monotonic() - recorded:.1f}s after recording its devices, "
                                    f"past half the ledger grace ({LEDGER_GRACE_S:.0f}s); rolled back for kube-scheduler to retry")
            self.api.bind_pod(namespace, name, uid, node)
            self.cache.bound(node, key)
        except Exception:
            self.cache.forget(node, key)
            try:  # roll back the annotation so a retry starts clean
                self.api.patch_pod_annotations(namespace, name, {ANN_GROUP: None, ANN_ASSIGNED: None, ANN_ASSUME_TIME: None,
                                                                 self.cfg.contract.cpuset_key: None})
            except Exception as e2:  # pragma: no cover - best effort
                log.warning("rollback of %s/%s annotations failed: %s", namespace, name, e2)
            if self.cfg.ledger:
                self._ledger_release(node, key)
            raise
        self.metrics.bound(d)
        log.info("bound %s to %s devices %s score %.2f (%s)", key, node, list(d.ids), d.score, d.policy)
        if self.cfg.events:
            record_event(self.api, pod, "GPUTopologyBound",
                         f"assigned devices {list(d.ids)} on {node} (score {d.score:.2f}, {d.policy})",
                         component="gpu-topology-extender")
        return d

    def _ledger_release(self, node: str, key: str, attempts: int = 4) -> None:
        """Drop ``key``'s ledger entry after a failed bind (best effort; the entry also lapses on its own
        once older than the grace period with no such pod on the node)."""
        for _ in range(attempts):
            try:
                self.ledger.release(self.api, node, key)
                return
            except Conflict:
                continue
            except Exception as e:  # noqa: BLE001 - best effort
                log.warning("releasing the ledger entry of %s on %s failed: %s", key, node, e)
                return

    def preempt(self, pod: Dict[str, Any], victims: Dict[str, Tuple[List[str], int]],
                max_subsets: int = 4096) -> Dict[str, Tuple[List[str], int]]:
        """kube-scheduler extender ``preemptVerb``: refine the scheduler's victims per candidate node.

        kube-scheduler picks victims by priority and resource counts only; any lower-priority pods that
        together free k devices qualify, wherever those devices sit.  Here, per node, the victims that
        hold no GROUP devices (chosen for CPU/memory, or holding devices without an annotation) are kept
        as proposed, and among the GROUP holders the extender keeps the smallest subset whose devices,
        together with the free ones, host the pod — and among those the one whose best placement has
        the lowest objective (evicting the two pods on one NUMA half beats evicting one on each).
        Nodes where even all victims do not make the pod placeable are dropped.  ``victims``:
        node -> (victim pod UIDs, NumPDBViolations); the PDB count is passed through (fewer victims
        can only violate fewer budgets)."""
        import itertools

        t0 = time.perf_counter()
        try:
            k = self.request_of(pod)
        except MalformedPod:
            return dict(victims)  # not ours to judge: kube-scheduler's own victims stand
        out: Dict[str, Tuple[List[str], int]] = {}
        shape, _ = self._pod_shape(pod, k) if k else (None, "")
        for node, (uids, pdb) in victims.items():
            if k == 0:
                out[node] = (list(uids), pdb)
                continue
            if shape is None:
                continue
            st = self.cache.get(node)
            with st.lock:
                t = st.topology
                now = self.clock()
                if t is None or st.probing_until > now:  # a node being re-probed is not a candidate either
                    continue
                live = {a.uid: a for a in st.allocs.values()
                        if a.uid and (a.assigned or now - a.assume_time <= self.cfg.assume_ttl)}
                gpu = [u for u in uids if u in live]
                keep = [u for u in uids if u not in live]
                freed_unknown = sum(st.unknown_pods.get(st.unknown_uids.get(u, ""), 0) for u in keep)
                used = st.used(now, self.cfg.assume_ttl)
                healthy = {g.index for g in t.gpus if g.healthy}
                _, fraction, numa, _, multi, mem, unit, steps = shape
                if not self._pool_ok(t, unit)[0]:
                    continue
                tm = tm_from_labels(st.labels, self.cfg.contract.prefix)
                if fraction == 0.0 and mem is not None and len({g.physical for g in t.gpus}) == t.n:
                    fraction = None  # memory-sized request on whole GPUs: an ordinary placement
                access = access_costs(t, numa) if self.cfg.cpu_affinity else None
                best = None
                tried = 0
                for r in range(0, len(gpu) + 1):
                    for sub in itertools.combinations(gpu, r):
                        tried += 1
                        if tried > max_subsets:
                            break
                        freed = set().union(*(live[u].ids for u in sub)) if sub else set()
                        still = sorted((used - freed) & set(range(t.n)))
                        free = len(healthy) - len(set(still) & healthy) - max(0, st.unknown - freed_unknown)
                        if free < k:
                            continue
                        try:
                            if tm.active and fraction is None and steps:
                                # the kubelet's Topology Manager must admit the pod on what the victims free
                                ids, _ = self._choose_aligned(t, still, k, access, multi, steps, tm)
                                if ids is None:
                                    continue
                                _, obj = self._rate(t, still, ids, access, multi)
                            else:
                                _, _, obj = self._choose_cached(t, still, k, access, fraction, multi)
                        except NoFeasiblePlacement:
                            continue
                        if best is None or obj < best[0] - 1e-12:
                            best = (obj, list(sub))
                    if best is not None or tried > max_subsets:
                        break  # the smallest victim count that works (or the search budget) decides
                if best is None:
                    continue
                chosen = set(best[1])
                out[node] = ([u for u in uids if u in chosen or u in keep], pdb)
        self.metrics.observe("preempt", time.perf_counter() - t0)
        return out

    def defrag(self, k: int, max_moves: int = 3, min_score: float = 0.0) -> Optional[Dict[str, object]]:
        """Operator view (``GET <prefix>/defrag?gpus=k``, ``gtk defrag``): the fewest pod moves after
        which a ``k``-device pod fits well on some node (:func:`placement.defrag.plan_defrag`), planned
        on the cache's current view.  Nodes carrying pods whose devices are unknown (no GROUP
        annotation) are left out: their used sets are not exact."""
        from ..placement.defrag import plan_defrag

        if self.cache.informer is None:
            self.cache.sync_all()
        elif not self.cache.informed():
            return None  # still listing: no plan from a partial view, and no cluster LIST per request
        now = self.clock()
        nodes: Dict[str, Topology] = {}
        pods: Dict[str, Dict[str, Tuple[int, ...]]] = {}
        for st in self.cache.nodes():
            name = st.name
            with st.lock:
                if st.topology is None or st.unknown:
                    continue
                nodes[name] = st.topology
                pods[name] = {a.pod: tuple(a.ids) for a in st.allocs.values()
                              if a.assigned or now - a.assume_time <= self.cfg.assume_ttl}
        plan = plan_defrag(nodes, pods, k, self.cfg.policy, max_moves=max_moves, min_score=min_score)
        return None if plan is None else plan.to_dict()

    def _patch_with_retry(self, namespace: str, name: str, ann: Dict[str, str]) -> None:
        last: Optional[Exception] = None
        for attempt in range(max(1, self.cfg.bind_retries)):
            try:
                self.api.patch_pod_annotations(namespace, name, ann)
                return
            except ApiError as e:
                last = e
                if e.code < 500 and e.code != 409:
                    raise
                time.sleep(0.01 * (2**attempt))
        assert last is not None
        raise last
