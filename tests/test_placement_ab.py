"""The placement A/B made interpretable (paper p.7 Figs. 11-12, default
Kubernetes vs Gaia; ``design.md:11``): every compared subset — the scheduler's choice, the worst one and
the devices the kubelet hands out with no extender — comes with the objective's terms, what separates
it from the choice, and the gain its slowest link predicts."""
import json
import os
import subprocess
import sys

import pytest

from gpu_topology_on_k8s_amd.placement import select, worst
from gpu_topology_on_k8s_amd.placement.explain import TERMS, default_subset, explain_subsets
from gpu_topology_on_k8s_amd.topology import fixtures as fx

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _three(topo, k):
    return explain_subsets(topo, {"chosen": list(select(topo, k).ids), "worst": list(worst(topo, k).ids),
                                  "default": default_subset(topo, k)})


@pytest.mark.parametrize("k", [2, 4])
def test_healthy_mesh_predicts_no_link_gain(k):
    """Every xGMI link alike: the worst subset differs only by host-side terms (NUMA span, packing), so
    the predicted all-reduce gain is 1.00 — what the first k >= 2 run will print, explained."""
    ex = _three(fx.f7_mi355x(link_gbps=150.0), k)
    assert ex["chosen"]["objective"] <= ex["default"]["objective"] <= ex["worst"]["objective"]
    vs = ex["vs_worst"]
    assert not vs["link_terms_separate"] and vs["predicted_gain"] == pytest.approx(1.0)
    assert set(vs["separating_terms"]) <= {"span", "frag", "fit", "access"} and vs["separating_terms"]
    assert ex["vs_default"]["same_devices"]  # on an empty node the kubelet's lowest ids are the choice too
    assert set(ex["chosen"]["weighted"]) == set(TERMS)


@pytest.mark.parametrize("k", [2, 4])
def test_degraded_link_separates_the_default_placement(k):
    """Link 0-1 at 60 %: the kubelet's lowest ids use it, the choice does not; the comparison names the
    link terms and predicts the slowest-link ratio, 1 / 0.6.  With four devices the ring-order bound is
    1.00: a ring 0-2-1-3-0 avoids the slow link, if RCCL's ring order does."""
    t = fx.f7_degraded(((0, 1, 0.6),))
    ex = _three(t, k)
    chosen, dflt = ex["chosen"]["ids"], ex["default"]["ids"]
    assert not {0, 1} <= set(chosen) and {0, 1} <= set(dflt)
    vs = ex["vs_default"]
    assert vs["link_terms_separate"] and "comm" in vs["separating_terms"]
    assert vs["predicted_gain"] == pytest.approx(1 / 0.6, rel=1e-3) and vs["predicted_basis"] == "slowest measured link"
    if k == 2:
        assert vs["predicted_gain_ring"] == pytest.approx(vs["predicted_gain"])
    else:
        assert vs["predicted_gain_ring"] == pytest.approx(1.0)
        assert ex["default"]["ring_link_gbps"] == pytest.approx(150.0) and ex["default"]["min_link_gbps"] == pytest.approx(90.0)
    assert ex["chosen"]["objective"] < ex["default"]["objective"]
    assert vs["predicted_gain"] >= ex["vs_worst"]["predicted_gain"] >= 1.0 - 1e-9


def _bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True, timeout=timeout,
                       cwd=REPO, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("n,fixture", [(2, "f7"), (4, "f7"), (2, "degraded"), (4, "degraded")])
def test_bench_dry_run_reports_three_subsets_with_terms(tmp_path, n, fixture):
    """gloo dry runs of the north-star line at N=2 and N=4 on F7 and on the one-degraded-link node: the
    line carries chosen / worst / default with their terms and predicted gains; where the kubelet's
    choice differs, it is timed as a third arm."""
    t = fx.f7_mi355x(link_gbps=150.0) if fixture == "f7" else fx.f7_degraded(((0, 1, 0.6),))
    path = tmp_path / "topo.json"
    path.write_text(t.to_json())
    out = _bench("--gpus", str(n), "--backend", "cpu", "--steps", "2", "--warmup", "1", "--size-mb", "1", "--sweep", "off",
                 "--cpu-visible", "8", "--topology-json", str(path))
    pt = out["placement_terms"]
    assert {"chosen", "worst", "default", "vs_worst", "vs_default"} <= set(pt)
    assert pt["chosen"]["ids"] == out["config"]["subset"]
    for name in ("chosen", "worst", "default"):
        assert set(pt[name]["weighted"]) == set(TERMS) and pt[name]["link_classes"] == ["XGMI"]
    assert out["worst_subset_ab"] and out["worst_subset_ab"]["exact"]
    if fixture == "f7":
        assert pt["vs_default"]["same_devices"] and out["config"]["default_subset"] is None and out["default_subset_ab"] is None
        assert pt["vs_worst"]["predicted_gain"] == pytest.approx(1.0)
    else:
        assert out["config"]["default_subset"] == pt["default"]["ids"]
        ab = out["default_subset_ab"]
        assert ab and ab["exact"] and ab["subset"] == out["config"]["default_subset"] and out["placement_gain_vs_default"] > 0
        assert pt["vs_default"]["predicted_gain"] == pytest.approx(1 / 0.6, rel=1e-3)
        assert pt["vs_default"]["predicted_gain_ring"] == pytest.approx(1 / 0.6 if n == 2 else 1.0, rel=1e-3)


def test_ring_cannot_route_round_two_slow_links_of_one_device():
    """Device 0 at 60 % toward both 1 and 2: any ring through {0,1,2,3} uses two of 0's three links, so
    one slow link is unavoidable and even the ring-order bound is 1 / 0.6."""
    t = fx.f7_degraded(((0, 1, 0.6), (0, 2, 0.6)))
    ex = _three(t, 4)
    assert {0, 1, 2, 3} == set(ex["default"]["ids"]) and 0 not in ex["chosen"]["ids"]
    assert ex["default"]["ring_link_gbps"] == pytest.approx(90.0)
    assert ex["vs_default"]["predicted_gain"] == pytest.approx(1 / 0.6, rel=1e-3)
    assert ex["vs_default"]["predicted_gain_ring"] == pytest.approx(1 / 0.6, rel=1e-3)


def test_ring_bound_model():
    """The ring bound on hand-made speeds: every pair for k <= 3, the best ring's slowest link for 4..8."""
    import itertools

    import numpy as np

    from gpu_topology_on_k8s_amd.placement.explain import _ring_bound

    def sp(k, slow):
        m = np.full((k, k), 2.0)
        for a, b in slow:
            m[a, b] = m[b, a] = 1.0
        return m

    assert _ring_bound(sp(3, [(0, 1)])) == 1.0
    assert _ring_bound(sp(4, [(0, 1)])) == 2.0
    assert _ring_bound(sp(4, [(0, 1), (2, 3), (0, 2)])) == 1.0  # 2's only fast link left is 2-1: a ring needs two
    assert _ring_bound(np.zeros((1, 1))) is None
    # against a plain enumeration, on random speeds for 4..8 devices
    rng = np.random.default_rng(0)
    for k in range(4, 9):
        m = rng.uniform(1, 2, (k, k))
        m = np.minimum(m, m.T)
        want = max(min(m[x, y] for x, y in zip((0,) + p, p + (0,))) for p in itertools.permutations(range(1, k)))
        assert _ring_bound(m) == want


def test_train_harness_runs_the_default_arm(tmp_path):
    """bench/train_llama.py on a degraded fake node (CPU, 2 ranks): best, worst and the kubelet's default
    are three different device sets, each trained, and the summary carries the terms."""
    t = fx.f7_degraded(((0, 1, 0.6),))
    path = tmp_path / "topo.json"
    path.write_text(t.to_json())
    out = tmp_path / "r.json"
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench", "train_llama.py"), "--gpus", "2", "--device", "cpu",
                        "--discovery", "fake", "--model", "tiny", "--batch", "1", "--seq", "64", "--steps", "2", "--warmup", "1",
                        "--attn", "sdpa", "--gemm-tuning", "off", "--topology-json", str(path), "--out", str(out)],
                       capture_output=True, text=True, timeout=900, cwd=REPO, env=dict(env, GTK_FAKE_GPUS="8"))
    assert p.returncode == 0, p.stderr[-4000:]
    r = json.loads(out.read_text())
    s = r["summary"]
    assert set(r["runs"]) == {"best", "worst", "default"}
    assert s["default_devices"] == [0, 1] and not s["default_same_as_best"] and s["default_throughput"] > 0
    # the kubelet's lowest ids are the degraded pair, which is also the objective's worst: measured once
    assert r["runs"]["worst"]["devices"] == [0, 1] and s["default_same_as_worst"]
    assert len({tuple(r["runs"][k]["devices"]) for k in r["runs"]}) == 2
    assert s["placement_terms"]["vs_default"]["link_terms_separate"]
