"""Prometheus metrics of the extender: per-verb latency histograms, chosen-score
histogram, bind count, and cluster fragmentation gauges computed from the node cache at scrape
time.  Uses a private registry so several extenders can live in one process (tests, cluster
simulation).

Fragmentation index of a node = 1 - (free devices in its fullest group) / (free devices), where a
group is a physical GPU on partitioned nodes and a NUMA domain otherwise: 0 when every free device
sits in one group (the next large request gets a compact set), toward 1 as free devices scatter.
The cluster index weights nodes by free devices.  ``gtk_extender_placeable_nodes{k}`` counts the
nodes that can still host a k-device pod.

The informer's health (k8s/informer.py) is exported per kind: complete LISTs (a count above 1 is a
relist, which at 100,000 pods costs tens of seconds and hundreds of MB: ``profiles/sched/INFORMER.md``),
LIST pages, watch events, watches resumed and watch errors, and the size and duration of the last LIST."""
from __future__ import annotations

from typing import TYPE_CHECKING

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily

if TYPE_CHECKING:  # pragma: no cover
    from .scheduler import Decision

_LAT_BUCKETS = (1e-5, 3e-5, 1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 0.1, 0.3, 1.0, 3.0)


class ExtenderMetrics:
    def __init__(self):
        self.registry = CollectorRegistry()
        self.latency = Histogram("gtk_extender_verb_seconds", "extender verb latency", ["verb"], buckets=_LAT_BUCKETS,
                                 registry=self.registry)
        self.requests = Counter("gtk_extender_requests_total", "extender requests", ["verb", "outcome"], registry=self.registry)
        self.scores = Histogram("gtk_extender_placement_score", "placement score of feasible nodes (0..10)",
                                buckets=tuple(range(0, 11)), registry=self.registry)
        self.binds = Counter("gtk_extender_binds_total", "pods bound with a device group", ["devices"], registry=self.registry)
        self.select_us = Histogram("gtk_extender_select_microseconds", "placement search time at bind",
                                   buckets=(10, 30, 100, 300, 1000, 3000, 1e4, 3e4, 1e5, 1e6), registry=self.registry)

        self.decision_cache = Counter("gtk_extender_decision_cache_total", "placement decisions served from / added to the cache",
                                      ["result"], registry=self.registry)

        self.ledger_conflict = Counter("gtk_extender_ledger_conflicts_total",
                                       "binds whose node allocation ledger changed under them (409): re-decided",
                                       registry=self.registry)
        self.ledger_conflicts = 0
        self.bind_lock_seconds = Histogram("gtk_extender_bind_node_lock_seconds",
                                           "time a bind held its node's lock (refresh + decide + ledger + annotate + bind): "
                                           "informer events for that node wait this long",
                                           buckets=_LAT_BUCKETS + (10.0, 30.0), registry=self.registry)
        self.bind_aborts = Counter("gtk_extender_bind_aborts_total",
                                   "binds given up because they ran out of time (retry budget, or too slow to finish "
                                   "before their ledger entry could lapse in another extender's view)", ["reason"],
                                   registry=self.registry)
        for reason in ("budget", "ledger_grace"):  # exported at 0 from the start (the alerts use increase())
            self.bind_aborts.labels(reason)
        self.probing_skips = Counter("gtk_extender_probing_skips_total",
                                     "node evaluations skipped because the node's device plugin is re-probing its links",
                                     registry=self.registry)
        self._hit, self._miss = self.decision_cache.labels(result="hit"), self.decision_cache.labels(result="miss")
        self._cache = None

    def attach_cache(self, cache, ttl: float, clock) -> None:
        """Export fragmentation gauges from ``cache`` (an :class:`~.cache.ClusterCache`) at scrape time."""
        if self._cache is None:
            self.registry.register(_FragmentationCollector(cache, ttl, clock))
            self.registry.register(_InformerCollector(cache))
        self._cache = cache

    def cache(self, hit: bool, n: int = 1) -> None:
        (self._hit if hit else self._miss).inc(n)

    def observe(self, verb: str, seconds: float) -> None:
        self.latency.labels(verb).observe(seconds)

    def request(self, verb: str, outcome: str) -> None:
        self.requests.labels(verb, outcome).inc()

    def score(self, s: float) -> None:
        self.scores.observe(s)

    def bound(self, d: "Decision") -> None:
        self.binds.labels(str(len(d.ids))).inc()
        self.select_us.observe(d.micros)

    def exposition(self) -> bytes:
        return generate_latest(self.registry)


def node_fragmentation(topology, used, unknown: int = 0):
    """(free devices, fragmentation index in [0, 1], largest free group) of one node."""
    if topology is None:
        return 0, 0.0, 0
    partitioned = len({g.physical for g in topology.gpus}) < topology.n
    groups = {}
    free = 0
    for g in topology.gpus:
        if g.healthy and g.index not in used:
            key = g.physical if partitioned else g.numa
            groups[key] = groups.get(key, 0) + 1
            free += 1
    free = max(0, free - unknown)
    if free == 0:
        return 0, 0.0, 0
    big = min(free, max(groups.values()))
    return free, 1.0 - big / free, big


class _FragmentationCollector:
    def __init__(self, cache, ttl: float, clock):
        self.cache, self.ttl, self.clock = cache, ttl, clock

    def collect(self):
        node_g = GaugeMetricFamily("gtk_extender_node_fragmentation", "1 - largest free group / free devices", labels=["node"])
        free_g = GaugeMetricFamily("gtk_extender_node_free_devices", "schedulable free devices", labels=["node"])
        place_g = GaugeMetricFamily("gtk_extender_placeable_nodes", "nodes with at least k free devices", labels=["k"])
        cluster_g = GaugeMetricFamily("gtk_extender_cluster_fragmentation", "free-device weighted fragmentation index")
        share_g = GaugeMetricFamily("gtk_extender_gpu_share_used",
                                    "fraction of a physical GPU's partitions / time slices held (partitioned or time-sliced nodes)",
                                    labels=["node", "gpu"])
        now = self.clock()
        tot_free = tot_big = 0
        counts = {1: 0, 2: 0, 4: 0, 8: 0}
        for st in self.cache.nodes():
            with st.lock:
                if st.topology is None:
                    continue
                used = st.used(now, self.ttl)
                free, frag, big = node_fragmentation(st.topology, used, st.unknown)
                per: dict = {}
                for g in st.topology.gpus:
                    n_all, n_used = per.get(g.physical, (0, 0))
                    per[g.physical] = (n_all + 1, n_used + (g.index in used))
            if any(n > 1 for n, _ in per.values()):
                for gpu, (n, u) in sorted(per.items()):
                    share_g.add_metric([st.name, str(gpu)], u / n)
            node_g.add_metric([st.name], frag)
            free_g.add_metric([st.name], free)
            tot_free += free
            tot_big += big
            for k in counts:
                counts[k] += free >= k
        for k, c in counts.items():
            place_g.add_metric([str(k)], c)
        cluster_g.add_metric([], (1.0 - tot_big / tot_free) if tot_free else 0.0)
        yield from (node_g, free_g, place_g, cluster_g, share_g)


class _InformerCollector:
    """The cache's informer counters at scrape time (nothing while the cache polls)."""

    def __init__(self, cache):
        self.cache = cache

    def collect(self):
        inf = getattr(self.cache, "informer", None)
        if inf is None:
            return
        fams = [(CounterMetricFamily(f"gtk_extender_informer_{name}", help_, labels=["kind"]), getattr(inf, attr))
                for name, attr, help_ in (
                    ("lists", "lists", "complete LISTs (more than one per kind: relists after a 410 Gone)"),
                    ("list_pages", "pages", "LIST requests (limit/continue pages)"),
                    ("events", "events", "watch events handed to the cache"),
                    ("watch_resumes", "watch_resumes", "watches re-opened from the last resourceVersion (no relist)"),
                    ("watch_errors", "watch_errors", "watches that broke (connection reset, 5xx, 429)"))]
        for fam, per_kind in fams:
            for kind, v in sorted(per_kind.items()):
                fam.add_metric([kind], float(v))
        items = GaugeMetricFamily("gtk_extender_informer_last_list_items", "objects in the last complete LIST", labels=["kind"])
        secs = GaugeMetricFamily("gtk_extender_informer_last_list_seconds", "duration of the last complete LIST", labels=["kind"])
        for kind, ll in sorted(dict(inf.last_list).items()):
            items.add_metric([kind], ll.get("items", 0.0))
            secs.add_metric([kind], ll.get("seconds", 0.0))
        synced = GaugeMetricFamily("gtk_extender_informer_synced", "1 once every kind has listed")
        synced.add_metric([], 1.0 if inf.synced else 0.0)
        yield from [f for f, _ in fams]
        yield from (items, secs, synced)
