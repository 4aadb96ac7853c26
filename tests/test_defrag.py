"""Defragmentation planner (placement/defrag.py): the fewest pod moves after which a k-GPU pod fits,
through the planner, the extender's cache view, its HTTP endpoint and the CLI."""
import json
import subprocess
import sys

from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.extender.server import make_app
from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer, PodAssignment, serve_http
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.placement.defrag import plan_defrag
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.shares import time_slice

C = Contract()


def _nodes(n=2):
    return {f"n{i}": fx.f7_mi355x() for i in range(n)}


def test_no_moves_when_the_pod_already_fits():
    plan = plan_defrag(_nodes(), {"n0": {"a": (0, 1)}}, 8)
    assert plan.node == "n1" and plan.moves == [] and plan.ids == tuple(range(8))


def test_one_small_pod_moves_to_free_a_whole_node():
    # n0 holds a 1-GPU pod, n1 a 2-GPU and a 4-GPU pod: 9 GPUs free, no node with 8
    pods = {"n0": {"small": (3,)}, "n1": {"two": (0, 1), "four": (4, 5, 6, 7)}}
    plan = plan_defrag(_nodes(), pods, 8)
    assert plan.node == "n0" and plan.moved_devices == 1
    (m,) = plan.moves
    assert (m.pod, m.src, m.dst) == ("small", "n0", "n1") and len(m.dst_ids) == 1 and m.dst_ids[0] in (2, 3)


def test_infeasible_and_immovable():
    pods = {"n0": {"a": (0, 1, 2, 3)}, "n1": {"b": (0, 1, 2, 3)}}
    plan = plan_defrag(_nodes(), pods, 8)  # one 4-GPU pod joins the other: a whole node frees up
    assert plan.moved_devices == 4 and plan.moves[0].dst_ids == (4, 5, 6, 7)
    pods = {"n0": {"a": tuple(range(6))}, "n1": {"b": tuple(range(6))}}
    assert plan_defrag(_nodes(), pods, 8) is None  # 4 free GPUs in the whole cluster
    pods = {"n0": {"small": (3,)}, "n1": {"two": (0, 1), "four": (4, 5, 6, 7)}}
    assert plan_defrag(_nodes(), pods, 8, movable=["two"]) is None


def test_a_pod_that_fits_is_never_moved_for():
    """Two 2-GPU pods on different NUMA halves of n0 and n1 full: a 4-GPU pod still fits on n0
    (2,3,6,7), so the plan proposes no move."""
    pods = {"n0": {"a": (0, 1), "b": (4, 5)}, "n1": {"c": tuple(range(8))}}
    plan = plan_defrag(_nodes(), pods, 4)
    assert plan.moves == [] and plan.node == "n0"


def test_sliced_nodes_are_left_out():
    nodes = {"s": time_slice(fx.f7_mi355x(n=2), 4), "w": fx.f7_mi355x(n=2)}
    # the 1-GPU pod could only move to "s", whose devices are slices of another shape: no plan
    assert plan_defrag(nodes, {"w": {"a": (0,)}}, 2) is None
    assert plan_defrag(nodes, {}, 2).node == "w"


def test_extender_endpoint_and_cli():
    api = FakeAPIServer()
    for n in ("n0", "n1"):
        api.create_node(make_node(n, annotations=encode_node_annotations(fx.f7_mi355x(), C),
                                  capacity={C.resource_name: "8"}))
    for name, node, ids in (("small", "n0", [3]), ("two", "n1", [0, 1]), ("four", "n1", [4, 5, 6, 7])):
        api.create_pod(make_pod(name, gpus=len(ids), node=node, annotations=PodAssignment(ids, True, 1).to_annotations()))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    plan = ext.defrag(8)
    assert plan["node"] == "n0" and plan["moved_devices"] == 1 and plan["moves"][0]["pod"] == "default/small"

    import asyncio

    from aiohttp.test_utils import TestClient, TestServer

    async def go():
        async with TestClient(TestServer(make_app(ext))) as cl:
            r = await cl.get("/gputopology-scheduler/defrag?gpus=8")
            return await r.json()

    body = asyncio.run(go())
    assert body["plan"]["moves"][0]["to"] == "n1"

    srv, url = serve_http(api)
    try:
        p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "defrag", "-k", "8", "--apiserver", url],
                           capture_output=True, text=True, timeout=120)
    finally:
        srv.shutdown()
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout)["plan"]["node"] == "n0"


def test_min_score_plans_for_a_numa_local_set():
    """Two 1-GPU pods, one on each NUMA half of n0: a 4-GPU pod fits (1,2,3,5) but spans both halves;
    asking for the score of a NUMA-local set moves one small pod to n1 and frees 0-3."""
    from gpu_topology_on_k8s_amd.placement import select

    pods = {"n0": {"a": (0,), "b": (4,)}, "n1": {"c": tuple(range(6))}}
    assert plan_defrag(_nodes(), pods, 4).moves == []
    local = select(fx.f7_mi355x(), 4).score
    plan = plan_defrag(_nodes(), pods, 4, min_score=local)
    assert plan.node == "n0" and plan.moved_devices == 1 and plan.score >= local
    assert {fx.f7_mi355x().gpus[i].numa for i in plan.ids} == {plan.moves[0].src_ids[0] // 4}


def test_gtk_status_reports_usage_and_scores():
    api = FakeAPIServer()
    for n in ("n0", "n1"):
        api.create_node(make_node(n, annotations=encode_node_annotations(fx.f7_mi355x(), C), capacity={C.resource_name: "8"}))
    api.patch_node("n1", labels={C.partition_request_label: "CPX", f"{C.prefix}/topology-manager-policy": "single-numa-node"},
                   annotations={C.partition_failed_key: "CPX/-: compute partition CPX: 0000:05:00.0: permission denied",
                                C.cordon_key: "7"})
    api.create_pod(make_pod("a", gpus=2, node="n0", annotations=PodAssignment([0, 4], True, 1).to_annotations()))
    srv, url = serve_http(api)
    try:
        p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "status", "--apiserver", url, "--output", "json"],
                           capture_output=True, text=True, timeout=120)
        q = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "status", "--apiserver", url],
                           capture_output=True, text=True, timeout=120)
    finally:
        srv.shutdown()
    assert p.returncode == 0, p.stderr
    rows = {r["node"]: r for r in json.loads(p.stdout)}
    assert rows["n0"]["used"] == 2 and rows["n0"]["free"] == 6 and rows["n1"]["free"] == 8
    assert rows["n0"]["best_score"]["8"] is None
    assert q.returncode == 0 and q.stdout.splitlines()[0].startswith("NODE") and "n1" in q.stdout
    assert "gpu_share_used" not in rows["n0"]
    assert rows["n0"]["partition"] == "SPX/NPS1" and not rows["n0"]["probing"] and "partition_request" not in rows["n0"]
    assert rows["n1"]["partition_request"] == "CPX/-" and "permission" in rows["n1"]["partition_change_failed"]
    # the operator's cordon and the kubelet's Topology Manager: a single-numa-node kubelet can take at most
    # one NUMA node's 4 GPUs, so an 8-GPU pod has no score there
    assert rows["n1"]["cordoned"] == "7" and rows["n1"]["topology_manager"] == "single-numa-node/container"
    assert rows["n1"]["best_score"]["8"] is None and rows["n1"]["best_score"]["4"] is not None and rows["n0"]["unhealthy"] == []
    assert "cordoned 7" in q.stdout and "topology-manager single-numa-node/container" in q.stdout


def test_gtk_status_shares_on_a_sliced_node():
    api = FakeAPIServer()
    api.create_node(make_node("s", annotations=encode_node_annotations(time_slice(fx.f7_mi355x(n=2), 4), C),
                              capacity={C.resource_name: "8"}))
    api.create_pod(make_pod("q", gpus=1, node="s", annotations=PodAssignment([5], True, 1).to_annotations()))
    srv, url = serve_http(api)
    try:
        p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "status", "--apiserver", url, "--output", "json",
                            "--sizes", "1,4"], capture_output=True, text=True, timeout=120)
    finally:
        srv.shutdown()
    (row,) = json.loads(p.stdout)
    assert row["per_gpu"] == 4 and row["gpu_share_used"] == {"0": 0.0, "1": 0.25}
    assert row["resource"] == C.slice_resource and row["best_score"]["4"] is not None  # scored in its own pool
