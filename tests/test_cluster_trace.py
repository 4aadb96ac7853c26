"""bench/cluster_trace.py: the cluster-level simulation drives the real placement code.

A small trace (4 nodes, 400 jobs) must: finish every job, keep allocations disjoint and within each
node, give topology-aware placement no more link inflation than the kubelet's lowest-id default, and
reduce fragmentation waiting against kube-scheduler's spread."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))

import cluster_trace as ct  # noqa: E402

from gpu_topology_on_k8s_amd.placement import PlacementPolicy  # noqa: E402
from gpu_topology_on_k8s_amd.placement.core import node_packing_term  # noqa: E402


@pytest.fixture(scope="module")
def results():
    topos = ct.make_cluster(4, 2, seed=7)
    trace = ct.make_trace(400, 32, 0.9, 60.0, seed=7)
    return {p: ct.run(topos, trace, p, alpha=0.5) for p in ("exact", "k8s-spread")}


def test_every_job_runs_and_metrics_are_sane(results):
    for r in results.values():
        assert 0 < r["goodput"] <= r["utilization"] <= 1.0
        assert r["jct_mean_min"] > 0 and r["makespan_h"] > 0


def test_exact_beats_spread(results):
    ex, sp = results["exact"], results["k8s-spread"]
    assert ex["runtime_inflation_mean"] <= sp["runtime_inflation_mean"] + 1e-9
    assert ex["frag_wait_gpu_hours"] < sp["frag_wait_gpu_hours"]


def test_allocations_disjoint_under_churn():
    topos = ct.make_cluster(2, 1, seed=3)
    sim = ct.Sim(topos, "exact", 0.5)
    held = []
    for k in (4, 2, 1, 1, 8, 4, 2):
        pl = sim.place(k)
        if pl is None:
            continue
        n, ids = pl
        assert len(ids) == k and not (set(ids) & sim.used[n])
        sim.used[n] |= set(ids)
        held.append((n, ids))
    assert sum(len(i) for _, i in held) == sum(len(u) for u in sim.used)


def test_ring_link_factor_avoids_a_single_bad_link():
    t = ct.make_cluster(1, 0, seed=1)[0]
    import numpy as np

    bw = np.full((8, 8), 153.0)
    bw[0, 1] = bw[1, 0] = 76.5
    t.set_measured_bw(bw, {"method": "synthetic"})
    sim = ct.Sim([t], "exact", 0.5, link_model="ring")
    assert sim.link_factor(0, (0, 1, 2, 3)) == pytest.approx(1.0)  # ring 0-2-1-3-0 skips the bad link
    assert sim.link_factor(0, (0, 1)) == pytest.approx(2.0)
    sim_b = ct.Sim([t], "exact", 0.5, link_model="bottleneck")
    assert sim_b.link_factor(0, (0, 1, 2, 3)) == pytest.approx(2.0)


def test_node_packing_prefers_the_fuller_node():
    pp = PlacementPolicy()
    # a 2-GPU job: a node with 2 free (exact fit) ranks before a half-used node and an untouched one
    assert node_packing_term(2, 2, 8, pp) < node_packing_term(4, 2, 8, pp) < node_packing_term(8, 2, 8, pp)


def test_share_trace_sharing_beats_whole_gpus_under_a_backlog():
    """bench/share_trace.py: with fractional jobs in the trace and a standing backlog, time-sliced
    shares placed by Fragment best fit do more useful work per GPU-hour than whole-GPU allocation,
    never over-commit a GPU, and finish every job."""
    import share_trace as stx

    from gpu_topology_on_k8s_amd.topology.model import Topology

    topos = [Topology.full_mesh(n=8, numa_split=2, node_name=f"n{i}") for i in range(3)]
    trace = stx.make_trace(300, 24, 1.2, 60.0, seed=3)
    whole = stx.run(topos, trace, "whole", 4)
    best = stx.run(topos, trace, "shares-bestfit", 4)
    assert best["goodput"] > whole["goodput"] and best["jct_mean_min"] < whole["jct_mean_min"]
    assert best["allocated"] == pytest.approx(best["goodput"])  # shares hold exactly what the jobs asked for
    assert whole["allocated"] > whole["goodput"]  # a 0.25-GPU job held a whole GPU

    sim = stx.Sim(topos, "shares-bestfit", 4)
    a = sim.place(0.5)
    sim.nodes[a[0]].slot_used |= set(a[1])
    b = sim.place(0.25)  # best fit: onto the half-used GPU, not a fresh one
    assert b[0] == a[0] and {i // 4 for i in b[1]} == {i // 4 for i in a[1]}


def test_bench_scripts_compile_and_document_themselves():
    """Every bench/ script (GPU-only ones included: share_mnist, share_neighbor, train_llama...) byte-
    compiles and prints its usage without a GPU."""
    import glob
    import py_compile
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for path in sorted(glob.glob(os.path.join(root, "bench", "*.py"))):
        py_compile.compile(path, doraise=True)
    for name in ("share_mnist.py", "share_neighbor.py", "share_trace.py"):
        p = subprocess.run([sys.executable, os.path.join(root, "bench", name), "--help"], capture_output=True, text=True, timeout=60)
        assert p.returncode == 0 and "usage" in p.stdout.lower(), (name, p.stderr[-500:])


def test_weights_and_single_gpu_rule_options():
    """The ablation knobs (profiles/sched/ablation): ``--weights`` replaces objective weights and rejects
    unknown names; ``--single farthest`` gives exact's 1-GPU jobs the device farthest from the others."""
    pp = ct.policy_from("w_fit=0, w_frag=0.5")
    assert pp.w_fit == 0.0 and pp.w_frag == 0.5 and pp.w_span == PlacementPolicy().w_span
    with pytest.raises(SystemExit):
        ct.policy_from("bogus=1")
    with pytest.raises(SystemExit):
        ct.policy_from("exact_limit=5")  # not a weight
    topos = ct.make_cluster(2, 2, seed=3)
    sim = ct.Sim(topos, "exact", 0.5, "bottleneck", pp, single="farthest")
    (i,), _ = sim._choose_on(0, 1)
    c = topos[0].cost
    far = max(range(8), key=lambda d: sum(c[d, x] for x in range(8) if x != d))
    assert i == far
    trace = ct.make_trace(60, 16, 0.9, 60.0, seed=3)
    r = ct.run(topos, trace, "exact", 0.5, "bottleneck", pp, "farthest")
    assert r["jct_mean_min"] > 0 and r["runtime_inflation_mean"] >= 1.0
