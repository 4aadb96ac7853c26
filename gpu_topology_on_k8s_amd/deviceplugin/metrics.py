"""Prometheus metrics of the device plugin.

Allocations and their latency, device health and health transitions, kubelet registrations, and the
link probe (last probe time, measured link GB/s summary, re-probes and republishes).  A private
registry per plugin so several plugins can live in one process (tests, the cluster simulation);
:func:`serve_metrics` exposes it over HTTP (``--metrics-port``).
"""
from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Tuple

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

__all__ = ["PluginMetrics", "serve_metrics"]

_LAT_BUCKETS = (1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 0.1, 0.3, 1.0, 3.0)


class PluginMetrics:
    def __init__(self):
        r = self.registry = CollectorRegistry()
        self.allocations = Counter("gtk_plugin_allocations_total", "Allocate calls by outcome", ["outcome"], registry=r)
        self.allocate_seconds = Histogram("gtk_plugin_allocate_seconds", "Allocate latency (pod claim + response)",
                                          buckets=_LAT_BUCKETS, registry=r)
        self.allocated_devices = Counter("gtk_plugin_allocated_devices_total", "devices handed to containers", registry=r)
        self.preferred = Counter("gtk_plugin_preferred_allocations_total", "GetPreferredAllocation answers by source",
                                 ["source"], registry=r)
        self.healthy = Gauge("gtk_plugin_device_healthy", "1 if the device is advertised Healthy", ["device"], registry=r)
        self.health_transitions = Counter("gtk_plugin_health_transitions_total", "Healthy<->Unhealthy changes",
                                          ["device", "to"], registry=r)
        self.registrations = Counter("gtk_plugin_registrations_total", "successful kubelet registrations", registry=r)
        self.probe_ts = Gauge("gtk_plugin_last_probe_timestamp_seconds", "unix time of the published link probe", registry=r)
        self.link_gbps = Gauge("gtk_plugin_link_read_gbps", "measured p2p read GB/s over the published matrix", ["stat"],
                               registry=r)
        self.reprobes = Counter("gtk_plugin_reprobes_total", "idle-time link re-measurements by result", ["result"], registry=r)
        self.partition_changes = Counter("gtk_plugin_partition_changes_total",
                                         "operator-requested GPU partition switches by outcome (ok, failed, skipped, busy)",
                                         ["outcome"], registry=r)
        self.guarded = Counter("gtk_plugin_guarded_containers_total",
                               "containers holding part of a GPU given the vGPU guard (HBM cap + forced CU mask)", registry=r)
        self.gpu_events = Counter("gtk_plugin_gpu_events_total", "amdsmi GPU event notifications by kind", ["kind"], registry=r)
        self.node_publishes = Counter("gtk_plugin_node_publishes_total", "node annotation PATCHes by outcome", ["outcome"],
                                      registry=r)
        self.validations = Counter("gtk_plugin_placement_validations_total", "PreStartContainer RCCL validations by result",
                                   ["result"], registry=r)
        self.validate_seconds = Histogram("gtk_plugin_placement_validation_seconds", "PreStartContainer validation time",
                                          buckets=(0.5, 1, 2, 5, 10, 30, 60, 120), registry=r)
        self.reconciled = Counter("gtk_plugin_reconciled_pods_total",
                                  "pod GROUP annotations corrected to the kubelet's pod-resources truth", registry=r)
        self.container_claims = Counter(
            "gtk_plugin_container_claims_total",
            "per-container Allocate calls of multi-container pods and mismatches, by how they matched a pod "
            "(partial, final, resized, unannotated)", ["how"], registry=r)
        self.group_overridden = Counter(
            "gtk_plugin_group_overridden_total",
            "Allocate calls whose devices were not the pod's GROUP, recorded as the kubelet chose them: the extender "
            "bound devices the kubelet did not offer (a Topology Manager policy the plugin was not told about, CPU or "
            "memory manager hints)", registry=r)
        self.cordoned = Gauge("gtk_plugin_cordoned_devices", "devices the operator took out of service (<prefix>/cordoned-gpus)",
                              registry=r)
        # every label value an alert watches exists from the start at 0 (deploy/prometheus-rules.yaml):
        # increase() cannot see the first increment of a series that appears at 1
        for outcome in ("ok", "invalid", "unhealthy", "missing", "stale_layout", "switch_wait", "probe_yield"):
            self.allocations.labels(outcome)
        for result in ("ok", "failed"):
            self.validations.labels(result)
        self.annotation_bytes = Gauge("gtk_plugin_topology_annotation_bytes", "encoded size of the published node annotations",
                                      registry=r)

    def set_topology(self, topo) -> None:
        import numpy as np

        ts = (topo.probe or {}).get("ts")
        if ts:
            self.probe_ts.set(float(ts))
        for g in topo.gpus:
            self.healthy.labels(str(g.index)).set(1.0 if g.healthy else 0.0)
        bw = topo.bw_gbps
        if bw is None:
            return
        off = bw[~np.eye(topo.n, dtype=bool)] if topo.n > 1 else np.array([])
        off = off[np.isfinite(off)]
        if off.size:
            for stat, v in (("min", off.min()), ("median", float(np.median(off))), ("max", off.max())):
                self.link_gbps.labels(stat).set(float(v))

    def health(self, index: int, healthy: bool) -> None:
        self.healthy.labels(str(index)).set(1.0 if healthy else 0.0)
        self.health_transitions.labels(str(index), "Healthy" if healthy else "Unhealthy").inc()

    def exposition(self) -> bytes:
        return generate_latest(self.registry)


class _Handler(BaseHTTPRequestHandler):
    metrics: PluginMetrics = None  # type: ignore[assignment]

    def log_message(self, *a):  # quiet
        pass

    def do_GET(self):
        if self.path.split("?")[0] == "/metrics":
            body, ctype = self.metrics.exposition(), "text/plain; version=0.0.4; charset=utf-8"
        elif self.path.split("?")[0] == "/healthz":
            live = getattr(self.metrics, "liveness", None)
            ok, why = live() if live is not None else (True, "ok")
            if not ok:  # the DaemonSet's livenessProbe restarts a wedged plugin
                body = why.encode()
                self.send_response(503)
                self.send_header("Content-Type", "text/plain")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)
                return
            body, ctype = b"ok", "text/plain"
        else:
            self.send_response(404)
            self.end_headers()
            return
        self.send_response(200)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)


def serve_metrics(metrics: PluginMetrics, host: str = "127.0.0.1", port: int = 0) -> Tuple[ThreadingHTTPServer, str]:
    """Serve ``/metrics`` and ``/healthz`` in a daemon thread; returns (server, base URL)."""
    handler = type("PluginMetricsHandler", (_Handler,), {"metrics": metrics})
    srv = ThreadingHTTPServer((host, port), handler)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, name="devplugin-metrics", daemon=True).start()
    return srv, f"http://{host}:{srv.server_address[1]}"
