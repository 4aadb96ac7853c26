"""Placement core: exact search == brute force, score properties, native engine == Python, legacy formulas."""
import itertools
import math
import os
import random
import subprocess
import time

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from gpu_topology_on_k8s_amd._native import available, binary
from gpu_topology_on_k8s_amd.placement import (
    NoFeasiblePlacement, PlacementPolicy, Problem, design_farthest_single, design_greedy_select, evaluate,
    legacy_score, legacy_score_of_set, select, worst,
)
from gpu_topology_on_k8s_amd.placement.legacy import legacy_mark, legacy_score_literal
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.model import RefLinkClass

needs_native = pytest.mark.skipif(not available("_placement"), reason="_placement not built")


def _random_problem(rng: np.random.Generator, n: int) -> Problem:
    c = rng.uniform(0.25, 4.0, size=(n, n))
    c = np.triu(c, 1)
    c = c + c.T
    free = rng.random(n) > 0.25
    levels = [np.array([0 if i < n // 2 else 1 for i in range(n)])]
    if rng.random() < 0.5:
        levels.insert(0, np.arange(n) // 2)
    access = np.where(rng.random(n) < 0.5, 0.0, rng.uniform(0, 2, n))
    return Problem(cost=c, free=free, levels=levels, access=access)


def _brute(p: Problem, k: int, policy=PlacementPolicy()):
    free_ids = [i for i in range(p.n) if p.free[i]]
    best, bj = None, math.inf
    for comb in itertools.combinations(free_ids, k):
        j, _ = evaluate(p, comb, policy)
        if j < bj - 1e-9:
            best, bj = comb, j
    return best, bj


@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=2, max_value=10), st.integers(min_value=0, max_value=2**31 - 1))
def test_python_exact_matches_bruteforce(n, seed):
    rng = np.random.default_rng(seed)
    p = _random_problem(rng, n)
    nfree = int(p.free.sum())
    for k in range(1, nfree + 1):
        pl = select(p, k, engine="python")
        ids, bj = _brute(p, k)
        assert pl.ids == ids
        assert pl.objective == pytest.approx(bj)


@needs_native
@settings(max_examples=80, deadline=None)
@given(st.integers(min_value=2, max_value=12), st.integers(min_value=0, max_value=2**31 - 1))
def test_native_engine_matches_python(n, seed):
    rng = np.random.default_rng(seed)
    p = _random_problem(rng, n)
    for k in range(1, int(p.free.sum()) + 1):
        a = select(p, k, engine="native")
        b = select(p, k, engine="python")
        assert a.exact
        assert a.ids == b.ids, (k, a, b)
        assert a.objective == pytest.approx(b.objective)
        for key in ("comm", "span", "frag", "fit", "access"):
            assert a.terms[key] == pytest.approx(b.terms[key])


@needs_native
@settings(max_examples=60, deadline=None)
@given(st.integers(min_value=2, max_value=10), st.integers(min_value=0, max_value=2**31 - 1))
def test_native_random_tie_break_matches_python(n, seed):
    """Random tie-break on the native engine: same tie list, same draw as the Python enumeration.
    Costs are quantised to a few classes so most requests have many optima (the mesh case)."""
    rng = np.random.default_rng(seed)
    p = _random_problem(rng, n)
    c = np.triu(rng.integers(1, 3, size=(n, n)).astype(float), 1)
    p = Problem(cost=c + c.T, free=p.free, levels=p.levels, access=np.zeros(n))
    pol = PlacementPolicy(tie_break="random")
    for k in range(1, int(p.free.sum()) + 1):
        a = select(p, k, policy=pol, rng=random.Random(seed + k), engine="native")
        b = select(p, k, policy=pol, rng=random.Random(seed + k), engine="python")
        assert a.ids == b.ids, (k, a, b)
        assert a.objective == pytest.approx(b.objective)


@needs_native
def test_native_tie_list_on_mi355x_mesh():
    """Full xGMI mesh, nothing used: every 2-subset is optimal, listed lexicographically."""
    import gpu_topology_on_k8s_amd.placement.core as core

    t = fx.f7_mi355x(link_gbps=76.5)
    p = Problem.from_topology(t)
    mod = core._native_engine()
    r = mod.select(p.cost, p.free, [lv.astype(np.int64).tolist() for lv in p.levels], p.access, 2, collect_ties=True)
    py_ties = []
    best = math.inf
    for comb in itertools.combinations(range(8), 2):
        j, _ = evaluate(p, comb)
        if j < best - 1e-9:
            best, py_ties = j, [list(comb)]
        elif j <= best + 1e-9:
            py_ties.append(list(comb))
    assert r["ties"] == py_ties


@needs_native
def test_native_engine_sanitizer_selftest():
    """ASan/UBSan host build of the engine vs brute force."""
    exe = binary("engine_selftest")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 failures" in p.stdout


def test_score_range_and_direction():
    t = fx.f7_mi355x(link_gbps=76.5)
    for k in range(1, 9):
        pl = select(t, k)
        assert 0 <= pl.score <= 10
        assert 0 <= pl.k8s_score <= 10
    # a degraded link makes every set containing it score lower
    bw = t.bw_gbps.copy()
    bw[0, 1] = bw[1, 0] = 10.0
    t.set_measured_bw(bw)
    p = Problem.from_topology(t)
    j_bad, _ = evaluate(p, (0, 1))
    j_ok, _ = evaluate(p, (0, 2))
    assert j_bad > j_ok
    assert select(t, 2).ids != (0, 1)


def test_full_mesh_four_gpu_picks_one_numa_domain():
    t = fx.f7_mi355x()
    assert select(t, 4).ids in ((0, 1, 2, 3), (4, 5, 6, 7))


def test_two_concurrent_four_gpu_pods_are_disjoint_numa_halves():
    """BASELINE config 4: two 4-GPU pods land on disjoint NUMA halves."""
    t = fx.f7_mi355x(link_gbps=76.5, noise=0.02, seed=5)
    a = select(t, 4)
    b = select(t, 4, used=a.ids)
    assert not set(a.ids) & set(b.ids)
    assert {t.gpus[i].numa for i in a.ids} != {t.gpus[i].numa for i in b.ids}
    assert len({t.gpus[i].numa for i in a.ids}) == 1 and len({t.gpus[i].numa for i in b.ids}) == 1


def test_singular_packing_on_mi355x():
    """Gaia Singular generalised: a 1-GPU request goes next to an existing allocation."""
    t = fx.f7_mi355x()
    first = select(t, 1).ids
    second = select(t, 1, used=first).ids
    assert t.gpus[first[0]].numa == t.gpus[second[0]].numa
    # after 3 single pods on NUMA0, a 4-GPU request still finds the pristine NUMA1
    used = []
    for _ in range(3):
        used += list(select(t, 1, used=used).ids)
    assert {t.gpus[i].numa for i in used} == {0}
    assert select(t, 4, used=used).ids == (4, 5, 6, 7)


def test_cpx_whole_package_first():
    t = fx.f8_mi355x_cpx()
    pl = select(t, 8)
    assert len({t.gpus[i].physical for i in pl.ids}) == 1
    pl2 = select(t, 8, used=pl.ids)
    assert len({t.gpus[i].physical for i in pl2.ids}) == 1
    assert not set(pl.ids) & set(pl2.ids)


@needs_native
def test_cpx_large_requests_are_fast():
    t = fx.f8_mi355x_cpx(link_gbps=76.5, noise=0.05, seed=2)
    for k in (2, 4, 8, 16, 32):
        t0 = time.perf_counter()
        pl = select(t, k, used=[0, 9, 18])
        dt = time.perf_counter() - t0
        assert len(pl.ids) == k and not {0, 9, 18} & set(pl.ids)
        assert dt < 5.0, (k, dt)


def test_infeasible():
    t = fx.f7_mi355x()
    with pytest.raises(NoFeasiblePlacement):
        select(t, 5, used=[0, 1, 2, 3])
    with pytest.raises(ValueError):
        select(t, 0)


def test_unhealthy_devices_are_never_chosen():
    t = fx.f7_mi355x()
    t.gpus[0].healthy = False
    t.gpus[1].healthy = False
    assert not {0, 1} & set(select(t, 4).ids)
    assert not {0, 1} & set(select(t, 6).ids)


def test_random_tie_break_spreads():
    t = fx.f7_mi355x()
    rng = random.Random(1)
    pol = PlacementPolicy(tie_break="random")
    seen = {select(t, 1, policy=pol, rng=rng).ids for _ in range(200)}
    assert len(seen) > 1


def test_worst_is_worse_than_best():
    t = fx.f7_mi355x(link_gbps=76.5, noise=0.1, seed=9)
    for k in (2, 4, 6):
        assert worst(t, k).objective >= select(t, k).objective


# ------------------------------------------------------------------ reference (legacy) formulas
def test_design_example_score():
    """design.md:213-217: marks 1,1,1,2,3,3 -> 10*(1-11/36) = 6.94."""
    assert legacy_score([1, 1, 1, 2, 3, 3]) == pytest.approx(6.944, abs=1e-3)
    assert legacy_score([]) == 10.0  # single GPU
    # the literal typed formula multiplies by len -> negative nonsense
    assert legacy_score_literal([1, 1, 1, 2, 3, 3]) < 0


def test_legacy_marks():
    assert legacy_mark(RefLinkClass.SYS) == 1
    assert legacy_mark(RefLinkClass.PSB) == 6
    with pytest.raises(ValueError):
        legacy_mark(RefLinkClass.NV3)


def test_legacy_score_of_f1_set():
    t = fx.f1_nvlink_host()
    s = legacy_score_of_set(t, [0, 2, 4])  # all PHB (mark 3)
    assert s == pytest.approx(10 * (1 - 9 / 18))


def test_design_greedy_and_tie_flaw():
    t = fx.f1_nvlink_host()
    ids = design_greedy_select(t.cost, [], 2)
    assert t.ref_class[ids[0], ids[1]] == int(RefLinkClass.NV3)
    assert design_greedy_select(t.cost, [], 1) == [0]
    assert design_greedy_select(t.cost, list(range(7)), 2) == []
    # tie flaw (design.md:188-190): greedy can lock in a worse 3-set than the exact search
    d = np.array([[0, 1, 5, 5], [1, 0, 5, 5], [5, 5, 0, 1], [5, 5, 1, 0]], float)
    d[0, 2] = d[2, 0] = 1.2
    g = design_greedy_select(d, [], 3)
    gsum = sum(d[a, b] for a, b in itertools.combinations(g, 2))
    best = min(sum(d[a, b] for a, b in itertools.combinations(c, 2)) for c in itertools.combinations(range(4), 3))
    assert gsum >= best


def test_design_farthest_single():
    t = fx.f1_nvlink_host()
    i = design_farthest_single(t.cost, [])
    assert i is not None and 0 <= i < 8
    assert design_farthest_single(t.cost, list(range(8))) is None


def test_partition_aware_switch_on_cpx_node():
    """--partition-aware: with XCP grouping a 2-XCP request lands on one package (cheap
    on-package links); partition-blind treats every XCP as a stand-alone xGMI device."""
    from gpu_topology_on_k8s_amd.placement import PlacementPolicy, select
    from gpu_topology_on_k8s_amd.placement.core import Problem
    from gpu_topology_on_k8s_amd.topology.model import Topology

    t = Topology.full_mesh(n=2, partitions_per_gpu=4, numa_split=1)  # 2 GPUs x 4 XCPs
    aware = select(t, 2, used=[1, 2, 3], policy=PlacementPolicy(partition_aware=True))
    assert t.physical[list(aware.ids)].tolist() == [1, 1]
    blind_p = Problem.from_topology(t, [1, 2, 3], partition_aware=False)
    same = t.physical[:, None] == t.physical[None, :]
    off = ~np.eye(t.n, dtype=bool)
    assert np.allclose(blind_p.cost[same & off], blind_p.cost[~same].mean())  # on-package pairs priced as xGMI
    assert len(blind_p.levels) == 1  # NUMA only, no package level
    assert PlacementPolicy.from_dict(PlacementPolicy(partition_aware=False).to_dict()).partition_aware is False


@pytest.mark.parametrize("engine", ["python", "native"])
def test_bottleneck_term_avoids_a_slow_link_a_ring_cannot_skip(engine):
    """GPUs 5-7 are taken; links 0-1 and 0-2 run at a third of nominal.  Every ring over {0,1,2,3}
    uses one of them.  The mean pair cost alone (+2/3) keeps the job inside NUMA half 0-3 (crossing
    to GPU 4 costs w_span + w_frag = 0.75); the bottleneck term, or the link-deficit term, moves it to
    {1,2,3,4}."""
    if engine == "native" and not available("_placement"):
        pytest.skip("_placement not built")
    t = fx.f7_mi355x(link_gbps=76.5)  # cost 1.0 per nominal link
    bw = np.array(t.bw_gbps, dtype=float)
    for a, b in ((0, 1), (0, 2)):
        bw[a, b] = bw[b, a] = bw[a, b] / 3.0
    t.set_measured_bw(bw, {"method": "synthetic"})
    used = [5, 6, 7]
    assert set(select(t, 4, used=used, policy=PlacementPolicy(w_bottleneck=0.0, w_link_deficit=0.0), engine=engine).ids) == {0, 1, 2, 3}
    # either term alone moves it: the bottleneck (worst pair), or the deficit (worst pair against the best of its class)
    assert set(select(t, 4, used=used, policy=PlacementPolicy(w_link_deficit=0.0), engine=engine).ids) == {1, 2, 3, 4}
    assert set(select(t, 4, used=used, policy=PlacementPolicy(w_bottleneck=0.0), engine=engine).ids) == {1, 2, 3, 4}
    pl = select(t, 4, used=used, policy=PlacementPolicy(), engine=engine)
    assert set(pl.ids) == {1, 2, 3, 4}
    assert pl.terms["bottleneck"] == pytest.approx(pl.comm)


def _two_nic_node():
    """F7 with one RDMA NIC per socket (like the MI355X gpurun box): GPUs 0-3 -> nic0, 4-7 -> nic1."""
    t = fx.f7_mi355x()
    t.nics = [{"name": "mlx5_0", "state": "4: ACTIVE"}, {"name": "mlx5_1", "state": "4: ACTIVE"}]
    t.gpu_nic = [[1, 5] if i < 4 else [5, 1] for i in range(8)]
    return t


@pytest.mark.parametrize("engine", ["python", "native"])
def test_multi_node_pod_spreads_over_nic_domains(engine):
    """A 2-GPU member of a multi-node job gets one GPU per NIC domain (twice the network bandwidth);
    a single-node pod stays in one NUMA half.  On a node without NICs the flag changes nothing."""
    if engine == "native" and not available("_placement"):
        pytest.skip("_placement not built")
    t = _two_nic_node()
    local = select(t, 2, engine=engine)
    assert {i // 4 for i in local.ids} == {0} or {i // 4 for i in local.ids} == {1}
    multi = select(t, 2, engine=engine, nic_aware=True)
    assert {i // 4 for i in multi.ids} == {0, 1} and multi.terms["nic_deficit"] == 0
    # only one domain left with free devices: nothing to spread over, no penalty
    half = select(t, 2, used=[4, 5, 6, 7], engine=engine, nic_aware=True)
    assert set(half.ids) <= {0, 1, 2, 3} and half.terms["nic_deficit"] == 0
    assert select(fx.f7_mi355x(), 2, engine=engine, nic_aware=True).ids == select(fx.f7_mi355x(), 2, engine=engine).ids


def test_a_healthy_node_has_no_link_deficit_and_places_as_before():
    """The link-deficit term is 0 on a healthy (banded) node, and on one whose costs come from link
    classes: no placement changes there."""
    from gpu_topology_on_k8s_amd.placement.core import Problem

    for t in (fx.f7_mi355x(link_gbps=150.0), fx.f7_mi355x(), fx.f8_mi355x_cpx()):
        assert Problem.from_topology(t).deficit is None
    t = fx.f7_mi355x(link_gbps=150.0)
    for k in (1, 2, 3, 4, 5, 8):
        for used in ([], [0], [4, 5, 6], [1, 2, 6]):
            if 8 - len(used) < k:
                continue
            a = select(t, k, used=used, engine="python")
            b = select(t, k, used=used, policy=PlacementPolicy(w_link_deficit=0.0), engine="python")
            assert a.ids == b.ids and a.objective == pytest.approx(b.objective)


@pytest.mark.parametrize("engine", ["python", "native"])
def test_a_degraded_link_outweighs_numa_locality_for_a_pair(engine):
    """Only GPUs 0, 1 (NUMA 0) and 7 (NUMA 1) are free and link 0-1 runs at 60 %: a 2-GPU pod's one
    link is its all-reduce's bottleneck, so the healthy cross-NUMA pair wins.  Without the deficit term
    NUMA locality (span) kept the slow pair."""
    if engine == "native" and not available("_placement"):
        pytest.skip("_placement not built")
    t = fx.f7_degraded(((0, 1, 0.6),))
    used = [2, 3, 4, 5, 6]
    pl = select(t, 2, used=used, engine=engine)
    assert 7 in pl.ids and pl.terms["link_deficit"] == 0.0
    assert select(t, 2, used=used, policy=PlacementPolicy(w_link_deficit=0.0), engine=engine).ids == (0, 1)
    assert worst(t, 2, used=used, engine=engine).ids == (0, 1)


def test_the_deficit_has_a_dead_band_and_keeps_link_classes_apart():
    from gpu_topology_on_k8s_amd.placement.core import LINK_DEFICIT_BAND, Problem

    for frac, want in ((0.95, 0.0), (0.85, 1 / 0.85 - 1 - LINK_DEFICIT_BAND), (0.5, 1.0 - LINK_DEFICIT_BAND)):
        d = Problem.from_topology(fx.f7_degraded(((2, 5, frac),))).deficit
        got = 0.0 if d is None else float(d[2, 5])
        assert got == pytest.approx(max(0.0, want), abs=1e-6), frac
        if d is not None:
            assert float(np.delete(np.delete(d, [2, 5], 0), [2, 5], 1).max()) == 0.0  # the healthy links: none


@pytest.mark.parametrize("seed", range(6))
def test_native_and_python_agree_with_degraded_links(seed):
    """Random noisy matrices with a few degraded links: the branch-and-bound engine (its deficit bound
    included) finds the Python enumeration's set and objective."""
    if not available("_placement"):
        pytest.skip("_placement not built")
    rng = np.random.default_rng(seed)
    t = fx.f7_mi355x(link_gbps=150.0)
    bw = np.array(t.bw_gbps, dtype=float) * (1 + rng.uniform(-0.04, 0.04, (8, 8)))
    for _ in range(3):
        a, b = rng.choice(8, 2, replace=False)
        bw[a, b] = bw[b, a] = 150.0 * rng.uniform(0.3, 0.85)
    np.fill_diagonal(bw, np.nan)
    t.set_measured_bw(bw, {"method": "synthetic"})
    for k in (2, 3, 4, 6):
        used = sorted(rng.choice(8, int(rng.integers(0, 8 - k + 1)), replace=False).tolist())
        a, b = select(t, k, used=used, engine="python"), select(t, k, used=used, engine="native")
        assert a.ids == b.ids and a.objective == pytest.approx(b.objective), (seed, k, used)
        assert a.terms["link_deficit"] == pytest.approx(b.terms["link_deficit"])
        wa, wb = worst(t, k, used=used, engine="python"), worst(t, k, used=used, engine="native")
        assert wa.objective == pytest.approx(wb.objective)
