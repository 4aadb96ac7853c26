"""Device health for ``ListAndWatch``.

The reference reports an ``isUsed`` bit per device and nothing about health (``design.md:84-86``,
diagram step ①).  Here the kubelet learns ``Unhealthy`` from the same RAS signals an operator would
look at, read by discovery (``csrc/topo/topo_reader.cpp``: amdsmi, or amdgpu sysfs ``ras/``):

* **uncorrectable ECC errors** — a count that grew since the plugin started (counts accumulate
  from driver load, so a device is judged by what happens on our watch, not by its history);
* **retired VRAM pages** at or over the driver's bad-page threshold (the driver is about to take
  the device out of service);
* **xGMI links** — fewer links up than at start (a link that drops mid-run forces RCCL onto slower
  paths and breaks the measured link-cost matrix the extender placed with);
* **vanished device** — discovery no longer lists it.

A device that recovers (e.g. links retrain) becomes Healthy again on the next poll.  Signals a node
cannot read (``-1``: unsupported, or no root) are ignored rather than treated as failures.

A lost xGMI link need not take the GPU out of service (``HealthPolicy(xgmi_links=False)``, the
daemon's ``--xgmi-link-loss degrade``): :meth:`HealthMonitor.relink` rebuilds the published model
with the re-discovered link class and hop count of every pair that changed, drops those pairs'
stale probe measurements, and the plugin republishes it — the extender then prices the pair at its
new class (e.g. PCIe across sockets, 8x a nominal xGMI link) and steers multi-GPU sets around it.
"""
from __future__ import annotations

import copy
import logging
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from ..topology.model import GPUInfo, Topology

log = logging.getLogger(__name__)

__all__ = ["HealthPolicy", "HealthMonitor", "device_problems"]


@dataclass(frozen=True)
class HealthPolicy:
    ecc_uncorrectable: bool = True
    bad_pages: bool = True
    xgmi_links: bool = True


def device_problems(now: GPUInfo, base: GPUInfo, policy: HealthPolicy = HealthPolicy()) -> List[str]:
    """Reasons ``now`` is unhealthy relative to its start-of-watch state ``base`` (empty = healthy)."""
    out: List[str] = []
    if not now.healthy:
        out.append("discovery reports the device unhealthy")
    if policy.ecc_uncorrectable and now.ecc_uncorrectable >= 0 and base.ecc_uncorrectable >= 0 \
            and now.ecc_uncorrectable > base.ecc_uncorrectable:
        out.append(f"uncorrectable ECC errors {base.ecc_uncorrectable} -> {now.ecc_uncorrectable}")
    if policy.bad_pages and now.bad_pages >= 0 and now.bad_page_threshold > 0 and now.bad_pages >= now.bad_page_threshold:
        out.append(f"retired pages {now.bad_pages} >= threshold {now.bad_page_threshold}")
    if policy.xgmi_links and now.xgmi_links_up >= 0 and base.xgmi_links_up > 0 and now.xgmi_links_up < base.xgmi_links_up:
        out.append(f"xGMI links up {base.xgmi_links_up} -> {now.xgmi_links_up}")
    return out


class HealthMonitor:
    """``health_fn`` of :class:`DevicePluginServer`: re-discovers the node and maps every device of the
    advertised topology to healthy / unhealthy, logging each transition with its reasons."""

    def __init__(self, baseline: Topology, discover_fn: Callable[[], Topology], policy: HealthPolicy = HealthPolicy()):
        self.base = {g.index: GPUInfo(**vars(g)) for g in baseline.gpus}
        self.discover_fn = discover_fn
        self.policy = policy
        self.reasons: Dict[int, List[str]] = {}
        self.last: Optional[Topology] = None  # the latest re-discovery

    def evaluate(self, fresh: Topology) -> Dict[int, Tuple[bool, List[str]]]:
        now = {g.index: g for g in fresh.gpus}
        out: Dict[int, Tuple[bool, List[str]]] = {}
        for idx, base in self.base.items():
            g = now.get(idx)
            probs = ["device vanished from discovery"] if g is None else device_problems(g, base, self.policy)
            out[idx] = (not probs, probs)
        return out

    def layout_changed(self) -> Optional[str]:
        """Why the device set itself changed since start (compute/memory partition switch, devices
        added or removed), or None.  The advertised device IDs no longer describe the node then: the
        plugin exits so its DaemonSet restarts it, and the new process re-discovers, re-probes (when
        idle) and re-registers with the kubelet."""
        fresh = self.last
        if fresh is None:
            return None
        before = [(g.bdf, g.partition, g.memory_partition) for g in self.base.values()]
        now = [(g.bdf, g.partition, g.memory_partition) for g in fresh.gpus]
        if len(before) != len(now):
            return f"device count {len(before)} -> {len(now)}"
        diff = [i for i, (a, b) in enumerate(zip(before, now)) if a != b]
        if diff:
            i = diff[0]
            return f"device {i}: {before[i]} -> {now[i]}" + (f" (+{len(diff) - 1} more)" if len(diff) > 1 else "")
        return None

    def relink(self, current: Topology) -> Optional[Topology]:
        """``current`` with the link class / hops of the last re-discovery wherever they changed (and
        those pairs' measurements dropped), or None when no pair changed."""
        fresh = self.last
        if fresh is None or fresh.n != current.n:
            return None
        changed = (fresh.link_type != current.link_type) | (fresh.hops != current.hops)
        np.fill_diagonal(changed, False)
        if not changed.any():
            return None
        new = copy.deepcopy(current)
        new.link_type = fresh.link_type.copy()
        new.hops = fresh.hops.copy()
        bw = new.bw_gbps.copy()
        bw[changed] = np.nan
        pairs = [(int(i), int(j)) for i, j in zip(*np.nonzero(np.triu(changed)))]
        log.warning("link class changed for pairs %s: republishing without their stale measurements", pairs)
        new.set_measured_bw(bw, dict(new.probe, relinked=pairs) if new.probe else {"relinked": pairs})
        return new

    def __call__(self, topo: Topology) -> Dict[int, bool]:
        self.last = self.discover_fn()
        res = self.evaluate(self.last)
        for idx, (ok, probs) in res.items():
            if probs != self.reasons.get(idx, []):
                if probs:
                    log.warning("device %d unhealthy: %s", idx, "; ".join(probs))
                elif self.reasons.get(idx):
                    log.info("device %d healthy again", idx)
            self.reasons[idx] = probs
        return {idx: ok for idx, (ok, _) in res.items() if idx < topo.n}
