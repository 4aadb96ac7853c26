"""Full-mesh placement is decided by topology, not by probe noise.

On 8x MI355X every pair is one xGMI hop.  The probe measures every ordered pair ``repeats`` times; a
link within max(its repeat spread, its class's median spread, 3 %) of its link class's median takes
the class value (ops/checks.py ``band_links``).  Simulated here on fixture F7: each link has a
persistent offset of up to +-1 % and every repeat a further +-a % (a from 0 to 5 % by seed), five
repeats, median published.
"""
import numpy as np
import pytest

from gpu_topology_on_k8s_amd.ops.checks import apply_banding, band_links
from gpu_topology_on_k8s_amd.placement.core import select, worst
from gpu_topology_on_k8s_amd.topology.codec import encode_v2
from gpu_topology_on_k8s_amd.topology.fixtures import f7_mi355x

LINK = 77.0
SEEDS = range(50)


def _probe(seed, degraded=(), n=8, repeats=5):
    """(median matrix, spread matrix) of a simulated probe."""
    rng = np.random.default_rng(seed)
    amp = 0.05 * (seed % 11) / 10  # 0 .. 5 % per repeat
    raw = np.full((n, n), np.nan)
    spread = np.full((n, n), np.nan)
    for i in range(n):
        for j in range(n):
            if i == j:
                continue
            base = LINK * (1 + rng.uniform(-0.01, 0.01))
            if (min(i, j), max(i, j)) in degraded:
                base *= 0.8
            vals = base * (1 + rng.uniform(-amp, amp, repeats))
            med = float(np.median(vals))
            raw[i, j], spread[i, j] = med, (vals.max() - vals.min()) / med
    return raw, spread


def _banded(seed, degraded=()):
    t = f7_mi355x()
    raw, spread = _probe(seed, degraded)
    banded, rep = band_links(t, raw, spread)
    t.set_measured_bw(banded, {"raw_gbps": raw.tolist(), "spread": spread.tolist(), "banding": rep})
    return t, rep


def _reference(degraded=()):
    t = f7_mi355x()
    bw = np.full((8, 8), LINK)
    for a, b in degraded:
        bw[a, b] = bw[b, a] = LINK * 0.8
    np.fill_diagonal(bw, np.nan)
    t.set_measured_bw(bw, {"method": "exact"})
    return t


def _decisions(t):
    return [(select(t, k, engine="python").ids, worst(t, k, engine="python").ids) for k in range(1, 9)]


def test_noisy_full_mesh_places_like_the_noise_free_one():
    want = _decisions(_reference())
    for seed in SEEDS:
        t, rep = _banded(seed)
        assert rep["kept_count"] == 0, (seed, rep)
        off = t.bw_gbps[~np.eye(8, dtype=bool)]
        assert np.all(off == off[0]), seed  # every link the same number: cost ties are exact
        assert _decisions(t) == want, seed


def test_without_banding_noise_changes_the_choice():
    """The problem being solved: the raw medians of the same simulated probes do pick different sets."""
    want = _decisions(_reference())
    differ = 0
    for seed in range(10):
        t = f7_mi355x()
        raw, _ = _probe(seed)
        t.set_measured_bw(raw, {"method": "raw"})
        differ += _decisions(t) != want
    assert differ > 0


def test_a_degraded_link_is_still_avoided():
    bad = ((2, 5),)
    want = _decisions(_reference(bad))
    for seed in SEEDS:
        t, rep = _banded(seed, bad)
        assert sorted(map(tuple, rep["kept"])) == [(2, 5), (5, 2)], (seed, rep["kept"])
        assert t.bw_gbps[2, 5] < 0.85 * LINK
        got = _decisions(t)
        assert got == want, seed
        assert set(got[1][0]) != {2, 5}  # the best pair never is the slow one
        assert set(got[1][1]) == {2, 5}  # ... and it is the worst


def test_a_link_below_its_floor_keeps_its_number_even_inside_a_wide_band():
    t = f7_mi355x()
    raw, spread = _probe(3)
    raw[1, 6] = 30.0  # far below half the median: the pair floor (ops/checks.py)
    spread[1, 6] = 5.0  # a spread so wide that the band alone would snap it
    banded, rep = band_links(t, raw, spread)
    assert banded[1, 6] == 30.0 and [1, 6] in rep["kept"]
    # the class's own band can be that wide too (every repeat of a noisy probe spreading by 80 %): the
    # floor still keeps the slow link's number, it is not smoothed into the class's healthy value
    spread = np.where(np.isnan(spread), np.nan, 0.8)
    banded, rep = band_links(t, raw, spread)
    assert banded[1, 6] == 30.0 and [1, 6] in rep["kept"]
    assert banded[0, 1] == pytest.approx(np.nanmedian(raw[~np.eye(8, dtype=bool)]), rel=0.02)


def test_two_reprobes_of_one_node_publish_the_same_cost_annotation():
    first, _ = _banded(7)
    a1 = encode_v2(first)["m"]["bw_gbps"]
    for seed in (8, 9, 21, 42):
        t = f7_mi355x()
        raw, spread = _probe(seed)
        t.set_measured_bw(raw, {"raw_gbps": raw.tolist(), "spread": spread.tolist()})
        assert apply_banding(t, prev=first)
        assert all(c["reused_previous"] for c in t.probe["banding"]["classes"])
        assert encode_v2(t)["m"]["bw_gbps"] == a1, seed
        assert np.array_equal(t.cost, first.cost)


def test_a_changed_link_class_is_republished():
    """Hysteresis only within the band: a node whose links all got 10 % slower publishes new numbers."""
    first, _ = _banded(7)
    t = f7_mi355x()
    raw, spread = _probe(8)
    raw *= 0.9
    t.set_measured_bw(raw, {"raw_gbps": raw.tolist(), "spread": spread.tolist()})
    apply_banding(t, prev=first)
    assert not any(c["reused_previous"] for c in t.probe["banding"]["classes"])
    assert t.bw_gbps[0, 1] < 0.95 * first.bw_gbps[0, 1]


def test_banding_survives_the_annotation_round_trip():
    from gpu_topology_on_k8s_amd.topology.codec import decode_v2

    t, _ = _banded(5)
    back = decode_v2(encode_v2(t))
    assert np.array_equal(back.bw_gbps, t.bw_gbps, equal_nan=True)
    assert np.allclose(np.array(back.probe["raw_gbps"], dtype=float), np.array(t.probe["raw_gbps"], dtype=float),
                       rtol=1e-3, equal_nan=True)
    assert apply_banding(back, prev=t)
    assert np.array_equal(back.bw_gbps, t.bw_gbps, equal_nan=True)


@pytest.mark.parametrize("seed", [0, 10])
def test_partitioned_node_classes_are_banded_separately(seed):
    """On a CPX node (F8) the on-package XCP links are their own class: they are not snapped to the
    xGMI links' median."""
    from gpu_topology_on_k8s_amd.topology.fixtures import f8_mi355x_cpx

    t = f8_mi355x_cpx()
    n = t.n
    rng = np.random.default_rng(seed)
    raw = np.full((n, n), np.nan)
    for i in range(n):
        for j in range(n):
            if i != j:
                same = t.physical[i] == t.physical[j]
                raw[i, j] = (400.0 if same else LINK) * (1 + rng.uniform(-0.01, 0.01))
    banded, rep = band_links(t, raw, None)
    assert len(rep["classes"]) == 2 and rep["kept_count"] == 0
    same = t.physical[:, None] == t.physical[None, :]
    off = ~np.eye(n, dtype=bool)
    assert len(set(banded[same & off].tolist())) == 1 and len(set(banded[~same].tolist())) == 1


def test_a_link_whose_own_repeats_spread_widely_takes_its_band_from_them():
    """Class spread 1 % (band 3 %), one link 6 % below the class median whose own repeats spread 10 %:
    its median is as noisy as its offset, so it takes the class value; a link 6 % low with a tight 1 %
    spread is a real difference and keeps its measurement."""
    t = f7_mi355x()
    raw = np.full((8, 8), LINK)
    spread = np.full((8, 8), 0.01)
    np.fill_diagonal(raw, np.nan)
    raw[0, 1] = LINK * 0.94
    spread[0, 1] = 0.10
    raw[2, 3] = LINK * 0.94
    banded, rep = band_links(t, raw, spread)
    assert banded[0, 1] == pytest.approx(LINK) and banded[2, 3] == pytest.approx(LINK * 0.94)
    assert [2, 3] in rep["kept"] and [0, 1] not in rep["kept"]


def test_an_unstable_link_well_below_its_class_keeps_its_number():
    """ADVICE r5 (checks.py:161): a link at 60 % of its class whose repeats spread 45 % (an intermittently
    degraded link) is above the 0.5 x median floor, and its own spread alone would have widened its band
    to 45 %; the widening is capped, so it keeps its measured value and is reported unstable."""
    t = f7_mi355x()
    raw = np.full((8, 8), LINK)
    spread = np.full((8, 8), 0.01)
    np.fill_diagonal(raw, np.nan)
    raw[4, 6] = raw[6, 4] = LINK * 0.6
    spread[4, 6] = spread[6, 4] = 0.45
    banded, rep = band_links(t, raw, spread)
    assert banded[4, 6] == pytest.approx(LINK * 0.6) and banded[6, 4] == pytest.approx(LINK * 0.6)
    assert [4, 6] in rep["kept"] and [4, 6] in rep["unstable"] and rep["unstable_count"] == 2
    t = _with(t, banded)
    assert t.cost[4, 6] > t.cost[4, 5] * 1.5  # the published cost carries it: placements pay for the link


def _with(t, bw):
    t.set_measured_bw(bw, {"method": "banded"})
    return t


def test_links_inside_a_package_and_across_packages_are_separate_classes():
    """XCPs of one package talk over Infinity Fabric, others over xGMI: even when a backend reports both
    as one-hop links of the same type, they are banded against their own class medians, not mixed."""
    from gpu_topology_on_k8s_amd.topology.fixtures import f8_mi355x_cpx

    t = f8_mi355x_cpx()
    n = t.n
    t.link_type[:, :] = t.link_type.max()  # one type for every pair (a backend that cannot tell them apart)
    np.fill_diagonal(t.link_type, 0)
    t.hops[:, :] = 1
    np.fill_diagonal(t.hops, 0)
    rng = np.random.default_rng(3)
    same = np.equal.outer(t.physical, t.physical)
    raw = np.where(same, 400.0, 60.0) * (1 + rng.uniform(-0.01, 0.01, (n, n)))
    np.fill_diagonal(raw, np.nan)
    banded, _ = band_links(t, raw, np.full((n, n), 0.01))
    off = ~np.eye(n, dtype=bool)
    assert np.unique(np.round(banded[same & off], 6)).size == 1  # every intra-package link on its class value
    assert np.unique(np.round(banded[~same], 6)).size == 1
