"""Cluster-in-a-process integration: BASELINE configs 1-4 through the full 7-step flow, restart
recovery and fault injection (SURVEY.md §4 "Integration", §5.3)."""
import numpy as np

from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.discovery import fake_topology


def test_config1_two_fake_gpus_one_gpu_pod():
    """Config 1: kind-style node with 2 fake CPU-backed GPUs via the device plugin; pod requests 1."""
    with SimCluster({"kind-worker": fake_topology(2)}, resource="aliyun.com/gpu") as c:
        c.submit("p", 1)
        (r,) = c.schedule_pending()
        assert r.node == "kind-worker" and len(r.devices) == 1 and r.allocated == r.devices
        pa = c.assignment("p")
        assert pa.assigned and pa.group == list(r.devices)
        node = c.api.get_node("kind-worker")
        assert node["status"]["capacity"]["aliyun.com/gpu"] == "2"


def test_config2_pair_on_directly_linked_gpus():
    """Config 2: a 2-GPU pod gets a pair on one direct, healthy xGMI link (never the degraded one)."""
    t = fx.f7_mi355x(link_gbps=76.5, noise=0.02, seed=3)
    bw = t.bw_gbps.copy()
    bw[0, 1] = bw[1, 0] = 20.0  # a degraded link measured by the probe
    t.set_measured_bw(bw)
    with SimCluster({"n": t}) as c:
        c.submit("pair", 2)
        (r,) = c.schedule_pending()
        assert set(r.devices) != {0, 1}
        assert t.gpus[r.devices[0]].numa == t.gpus[r.devices[1]].numa
        assert t.hops[r.devices[0], r.devices[1]] == 1


def test_config3_four_clique_best_score():
    t = fx.f7_mi355x(link_gbps=76.5, noise=0.05, seed=11)
    with SimCluster({"n": t}) as c:
        c.submit("four", 4)
        (r,) = c.schedule_pending()
        assert len(r.devices) == 4 and len({t.gpus[i].numa for i in r.devices}) == 1
        assert r.score >= 8


def test_config4_two_concurrent_four_gpu_pods():
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 4)
        c.submit("b", 4)
        ra, rb = c.schedule_pending(concurrent=True)
        assert ra.node == rb.node == "n"
        assert {frozenset(ra.allocated), frozenset(rb.allocated)} == {frozenset(range(4)), frozenset(range(4, 8))}
        c.submit("c", 1)
        (rc,) = c.schedule_pending()
        assert rc.node is None  # full


def test_packing_across_nodes_and_release():
    with SimCluster({"n1": fx.f7_mi355x(), "n2": fx.f7_mi355x()}) as c:
        for i in range(3):
            c.submit(f"s{i}", 1)
        rs = c.schedule_pending()
        assert {r.node for r in rs} == {"n1"}  # singles pack onto one node (Gaia Singular spirit)
        c.submit("big", 8)
        (rb,) = c.schedule_pending()
        assert rb.node == "n2"
        for i in range(3):
            c.complete(f"s{i}")
        assert c.used_devices("n1") == []


def test_extender_restart_recovers_from_annotations():
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 4)
        (ra,) = c.schedule_pending()
        c.restart_extender()
        c.submit("b", 4)
        (rb,) = c.schedule_pending()
        assert not set(ra.devices) & set(rb.devices)


def test_kubelet_restart_plugin_reregisters_and_keeps_serving():
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        n = c.nodes["n"]
        n.kubelet.restart()
        import time

        t0 = time.time()
        while n.plugin.registered < 2 and time.time() - t0 < 10:
            time.sleep(0.05)
        n.kubelet.wait_for(c.resource)
        c.submit("a", 2)
        (r,) = c.schedule_pending()
        assert r.node == "n" and len(r.allocated) == 2


def test_apiserver_faults_on_bind_are_survivable():
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 2)
        c.api.inject("bind_pod", 500, times=1)
        (r,) = c.schedule_pending()
        assert r.node is None and "500" in r.error
        assert c.assignment("a") is None  # rolled back
        (r2,) = c.schedule_pending()  # the scheduler's retry succeeds
        assert r2.node == "n" and len(r2.allocated) == 2


def test_unhealthy_gpu_is_not_scheduled():
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.nodes["n"].plugin.set_health(2, False)
        c.submit("a", 7)
        (r,) = c.schedule_pending()
        assert r.node == "n" and 2 not in r.allocated


def test_gaia_policy_reproduces_table4_end_to_end():
    """Paper Table IV through the whole stack: gpu2 busy, 2-GPU request -> gpu0&gpu1."""
    tr = fx.f4_tree()
    from gpu_topology_on_k8s_amd.topology.model import GPUInfo, LinkType, Topology

    cost = np.array([[tr.pair_cost(i, j) for j in range(4)] for i in range(4)], float)
    t = Topology(gpus=[GPUInfo(index=i, numa=[0, 0, 1, 1][i]) for i in range(4)], link_type=np.full((4, 4), int(LinkType.PCIE)),
                 hops=np.ones((4, 4), int), cost=cost)
    with SimCluster({"p4": t}, policy_name="gaia") as c:
        c.submit("busy", 1)
        (r0,) = c.schedule_pending()
        assert r0.allocated[0] in (2, 3)  # Table I: a cost-1 PIX GPU
        c.submit("pair", 2)
        (r1,) = c.schedule_pending()
        assert r1.allocated == (0, 1)  # Table IV


def test_scheduling_latency_is_milliseconds():
    """BASELINE target 2: far below Gaia's 2.53-3.56 s per scheduling (paper Fig. 10)."""
    with SimCluster({f"n{i}": fx.f7_mi355x() for i in range(4)}) as c:
        for i in range(16):
            c.submit(f"p{i}", [1, 2, 4, 1][i % 4])
        rs = c.schedule_pending()
        assert all(r.node for r in rs)
        assert max(r.sched_ms for r in rs) < 1000
        assert float(np.median([r.sched_ms for r in rs])) < 200
