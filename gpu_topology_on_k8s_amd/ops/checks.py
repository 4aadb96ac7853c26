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

**Banding** (:func:`band_links`).  On a full xGMI mesh every pair is one hop and
the links are interchangeable, yet the measured GB/s differ by a few percent of noise; with cost =
ref / GB/s that noise alone would pick the "best" pair, rank the worst subset and change the node
annotation at every re-probe.  The probe repeats every pair (``repeats`` per preset) and records
each link's spread; a link within max(its spread, its class's median spread, :data:`BAND_MIN`) of its
link class's median takes the class value, so noise-equivalent links become exactly equal (the placement engine's symmetry
breaking then decides, deterministically).  A link outside that band, or below its pair floor,
keeps its measured number: a degraded link is still seen.  Given the previously published matrix a
class keeps its previous value while the new median stays within the band of it, so a re-probe of a
healthy node republishes the same numbers (the same cost annotation).

Reference: ``/root/reference/design.md:11`` (a job using n GPUs gets affine GPUs),
``design.md:25-27`` (link discovery) and ``design.md:47`` (the link weights TODO); the checks make a
wrong link matrix fail loudly instead of steering placements.
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
BAND_MIN = 0.03  # links within 3 % of their class median (or within their own repeat spread) are equal
# a link's own repeat spread widens its band at most this far: an unstable link (repeats spreading by
# tens of percent, e.g. an intermittently degraded one) is never snapped onto its class's healthy value
BAND_SPREAD_CAP = 0.10

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


def link_class(topo: Topology, a: int, b: int) -> Tuple[int, int, bool]:
    """Links the probe should find interchangeable: same link type, same hop count, and both ends on
    one package or both on different packages (XCPs of one GPU talk over Infinity Fabric)."""
    return int(topo.link_type[a, b]), int(topo.hops[a, b]), int(topo.physical[a]) == int(topo.physical[b])


def band_links(topo: Topology, raw: np.ndarray, spread: Optional[np.ndarray] = None,
               prev: Optional[np.ndarray] = None) -> Tuple[np.ndarray, Dict[str, object]]:
    """``raw``: measured per-direction GB/s (n x n, nan = unmeasured); ``spread``: each link's relative
    repeat spread ((max - min) / median over the probe's repeats; nan / None = unknown, taken as 0);
    ``prev``: the previously published (banded) matrix, or None.  -> (banded matrix, report)."""
    n = topo.n
    raw = np.asarray(raw, dtype=np.float64)
    sp = np.zeros((n, n)) if spread is None else np.nan_to_num(np.asarray(spread, dtype=np.float64), nan=0.0)
    out = raw.copy()
    meas = {(a, b): float(raw[a, b]) for a in range(n) for b in range(n) if a != b and np.isfinite(raw[a, b]) and raw[a, b] > 0}
    floors = pair_floors(topo, meas)
    classes: Dict[Tuple[int, int, bool], List[Pair]] = {}
    for pr in meas:
        classes.setdefault(link_class(topo, *pr), []).append(pr)
    report: Dict[str, object] = {"band_min": BAND_MIN, "band_spread_cap": BAND_SPREAD_CAP, "classes": [], "kept": [],
                                 "unstable": []}
    for key in sorted(classes):
        prs = classes[key]
        med = float(np.median([meas[p] for p in prs]))
        cls_band = max(BAND_MIN, float(np.median([sp[p] for p in prs])))
        value, reused = med, False
        if prev is not None:
            pv = [float(prev[p]) for p in prs if np.isfinite(prev[p]) and prev[p] > 0]
            if pv:
                pmed = float(np.median(pv))
                if abs(med - pmed) <= cls_band * pmed:
                    value, reused = pmed, True
        snapped = 0
        for p in prs:
            # the class's typical repeat spread, or this link's own up to BAND_SPREAD_CAP
            band = max(cls_band, min(float(sp[p]), BAND_SPREAD_CAP))
            if float(sp[p]) > BAND_SPREAD_CAP:
                report["unstable"].append([int(p[0]), int(p[1])])
            if abs(meas[p] - med) <= band * med and meas[p] >= floors[p]:
                out[p] = value
                snapped += 1
            else:
                report["kept"].append([int(p[0]), int(p[1])])
        report["classes"].append({"link_type": key[0], "hops": key[1], "same_package": key[2], "links": len(prs),
                                  "median_gbps": round(med, 2), "value_gbps": round(value, 2), "snapped": snapped,
                                  "reused_previous": reused})
    report["kept_count"] = len(report["kept"])
    report["kept"] = report["kept"][:64]  # the node annotation carries this report: bounded
    report["unstable_count"] = len(report["unstable"])
    report["unstable"] = report["unstable"][:64]
    return out, report


def apply_banding(topo: Topology, prev: Optional[Topology] = None) -> bool:
    """Re-derive ``topo``'s published matrix from the raw per-link measurements its probe recorded
    (``probe["raw_gbps"]`` / ``probe["spread"]``), banded against ``prev``'s published matrix when
    given.  False (nothing changed) when the topology carries no raw measurements."""
    pr = topo.probe or {}
    if pr.get("raw_gbps") is None:
        return False
    raw = np.array([[np.nan if x is None else float(x) for x in row] for row in pr["raw_gbps"]], dtype=np.float64)
    sp = pr.get("spread")
    spread = None if sp is None else np.array([[np.nan if x is None else float(x) for x in row] for row in sp])
    pbw = prev.bw_gbps if (prev is not None and prev.bw_gbps is not None and prev.n == topo.n) else None
    banded, rep = band_links(topo, raw, spread, pbw)
    topo.set_measured_bw(banded, dict(pr, banding=rep))
    return True
