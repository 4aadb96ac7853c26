"""Self-validation of multi-GPU probe results.

The first 8-GPU run of the framework happens on a node the builder never sees, so its probe numbers
must carry their own sanity checks.  A check that only compares a link with its siblings cannot see a
failure that hits every link alike (peer access silently routed through host staging: every pair
uniformly at PCIe rate), and one that compares a gather with one link cannot see a gather that
serialises its sources.  These checks anchor to absolute rates:

* **Pair floor.** Every measured pair reaches half its link's rated per-direction rate and half the
  node's median pair.  The rated rate is amdsmi's maximum link bandwidth
  (``amdsmi_get_minmax_bandwidth_between_processors``, read at discovery into
  ``probe["amdsmi_max_bw_mbps"]``), taken as the bidirectional figure AMD quotes for xGMI (153.6 GB/s
  per MI355X link: BASELINE.md "Link rates"), so per direction it is half of it.  Without an amdsmi
  value the link class's nominal rate applies.
* **Gather.** An all-peer gather into one GPU (K5) loads k-1 links at once, so it must reach half of
  (k-1) x the median single-pair read.
* **Ring.** Every member pulling from all others at once (K6) must keep 60 % of the pair-sum bound
  (the sum of its single-pair reads), and cannot exceed it by more than 10 %.

Reference: ``/root/reference/design.md:11`` (a job using n GPUs gets affine GPUs) and
``design.md:25-27`` (link discovery); the checks make a wrong link matrix fail loudly instead of
steering placements.
"""
from __future__ import annotations

import statistics
from typing import Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np

from ..topology.model import LinkType, Topology

# nominal BIDIRECTIONAL rate per link class, GB/s, when amdsmi reports none (MI355X xGMI: 153.6;
# PCIe Gen5 x16: 2 x 64)
NOMINAL_BIDIR_GBPS = {int(LinkType.XGMI): 153.6, int(LinkType.PCIE): 128.0, int(LinkType.PCIE_SYS): 128.0}

PAIR_RATED_FRACTION = 0.5  # of the per-direction rated rate
PAIR_MEDIAN_FRACTION = 0.5
GATHER_FRACTION = 0.5  # of (k-1) x median single-pair read
RING_MIN_FRACTION = 0.6  # of the pair-sum bound
RING_MAX_FRACTION = 1.1

Pair = Tuple[int, int]


def rated_link_gbps(topo: Topology, a: int, b: int) -> Optional[float]:
    """Per-direction rated rate of the link between topology indices ``a`` and ``b`` (GB/s), or None
    when neither amdsmi nor the link class gives one (same device, on-package, unknown)."""
    mx = (topo.probe or {}).get("amdsmi_max_bw_mbps")
    if mx is not None:
        try:
            v = float(mx[a][b])
        except (IndexError, TypeError, ValueError):
            v = 0.0
        if v > 0:
            return v / 1000.0 / 2.0
    nominal = NOMINAL_BIDIR_GBPS.get(int(topo.link_type[a, b]))
    return None if nominal is None else nominal / 2.0


def pair_floors(topo: Topology, rates: Mapping[Pair, float]) -> Dict[Pair, float]:
    """Floor of every measured ordered pair (topology indices)."""
    med = statistics.median(rates.values()) if rates else 0.0
    out = {}
    for (a, b) in rates:
        rated = rated_link_gbps(topo, a, b)
        out[(a, b)] = max(PAIR_MEDIAN_FRACTION * med, PAIR_RATED_FRACTION * rated if rated else 0.0)
    return out


def check_pairs(topo: Topology, rates: Mapping[Pair, float]) -> List[str]:
    """Problems with measured pair rates (GB/s); empty when every pair passes its floor."""
    floors = pair_floors(topo, rates)
    probs = []
    for p, v in sorted(rates.items()):
        if not np.isfinite(v) or v < floors[p]:
            rated = rated_link_gbps(topo, *p)
            probs.append(f"pair {p[0]}->{p[1]}: {v:.1f} GB/s below its floor {floors[p]:.1f} "
                         f"(rated {rated if rated is not None else 'n/a'} GB/s per direction, "
                         f"median {statistics.median(rates.values()):.1f})")
    return probs


def matrix_rates(topo: Topology, devs: Optional[Sequence[int]] = None) -> Dict[Pair, float]:
    """The measured off-diagonal pairs of ``topo.bw_gbps`` over ``devs`` (default: every device)."""
    assert topo.bw_gbps is not None, "topology carries no measured matrix"
    devs = list(range(topo.n)) if devs is None else list(devs)
    return {(a, b): float(topo.bw_gbps[a, b]) for a in devs for b in devs if a != b}


def check_gather(gather_gbps: float, single_gbps: Sequence[float]) -> List[str]:
    """An all-peer gather from ``len(single_gbps)`` sources against their single-pair reads."""
    k1 = len(single_gbps)
    if k1 < 1:
        return []
    floor = GATHER_FRACTION * k1 * statistics.median(single_gbps)
    if gather_gbps < floor:
        return [f"gather from {k1} peers: {gather_gbps:.1f} GB/s below {floor:.1f} "
                f"({GATHER_FRACTION} x {k1} x median single pair {statistics.median(single_gbps):.1f}): "
                "the sources do not stream concurrently"]
    return []


def check_ring(ring_bound_gbps: float, pair_sum_gbps: float) -> List[str]:
    """The K6 concurrent ring against the pair-sum bound of the same subset."""
    probs = []
    if ring_bound_gbps < RING_MIN_FRACTION * pair_sum_gbps:
        probs.append(f"ring bound {ring_bound_gbps:.1f} GB/s below {RING_MIN_FRACTION} x pair-sum {pair_sum_gbps:.1f}")
    if ring_bound_gbps > RING_MAX_FRACTION * pair_sum_gbps:
        probs.append(f"ring bound {ring_bound_gbps:.1f} GB/s above {RING_MAX_FRACTION} x pair-sum {pair_sum_gbps:.1f}: "
                     "the single-pair reads under-measure the links")
    return probs
