"""Prometheus metrics of the extender: per-verb latency histograms, chosen-score
histogram, bind count.  Uses a private registry so several extenders can live in one process
(tests, cluster simulation)."""
from __future__ import annotations

from typing import TYPE_CHECKING

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

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

    def cache(self, hit: bool) -> None:
        self.decision_cache.labels(result="hit" if hit else "miss").inc()

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
