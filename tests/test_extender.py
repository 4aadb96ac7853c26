"""Scheduler extender: verbs, assume cache / TTL, concurrency, model quota, HTTP wire format."""
import asyncio
import threading
import time

import pytest
from aiohttp.test_utils import TestClient, TestServer

from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.extender.server import make_app
from gpu_topology_on_k8s_amd.k8s import ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GROUP, Contract, FakeAPIServer, PodAssignment
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx


class Clock:
    def __init__(self, t=1_700_000_000.0):
        self.t = t

    def __call__(self):
        return self.t


def _cluster(nodes=("n1",), topo_fn=fx.f7_mi355x, **cfg):
    api = FakeAPIServer()
    c = Contract()
    for n in nodes:
        t = topo_fn()
        api.create_node(make_node(n, labels={c.label_model: "MI355X"}, annotations=encode_node_annotations(t, c),
                                  capacity={c.resource_name: str(t.n)}))
    clock = Clock()
    ext = TopologyExtender(api, ExtenderConfig(**{"resync_s": 0.0, **cfg}), clock=clock)
    return api, ext, clock


def _submit(api, name, k, **kw):
    return api.create_pod(make_pod(name, gpus=k, **kw))


def _bind(api, ext, name, node="n1", ns="default"):
    pod = api.get_pod(ns, name)
    return ext.bind(ns, name, pod["metadata"]["uid"], node)


def test_prioritize_scores_and_infeasible_nodes():
    api, ext, _ = _cluster(nodes=("n1", "n2"))
    api.create_node(make_node("cpu-only"))
    pod = _submit(api, "p", 4)
    res = dict(ext.prioritize(pod, ["n1", "n2", "cpu-only"]))
    assert res["n1"] == res["n2"] and 1 <= res["n1"] <= 10
    assert res["cpu-only"] == 0


def test_bind_writes_reference_annotations():
    api, ext, clock = _cluster()
    _submit(api, "p", 2)
    d = _bind(api, ext, "p")
    pod = api.get_pod("default", "p")
    ann = pod["metadata"]["annotations"]
    assert pod["spec"]["nodeName"] == "n1"
    assert ann[ANN_GROUP] == ",".join(map(str, d.ids))
    assert ann[ANN_ASSIGNED] == "false"
    assert ann[ANN_ASSUME_TIME] == str(int(clock.t))
    assert ann[Contract().numa_key] in ("0", "1")  # both devices in one NUMA domain


def test_config4_two_concurrent_four_gpu_pods_disjoint():
    """BASELINE config 4: two concurrent 4-GPU pods land on disjoint NUMA halves."""
    api, ext, _ = _cluster()
    _submit(api, "a", 4)
    _submit(api, "b", 4)
    out = {}

    def go(n):
        out[n] = _bind(api, ext, n)

    ts = [threading.Thread(target=go, args=(n,)) for n in ("a", "b")]
    [t.start() for t in ts]
    [t.join() for t in ts]
    a, b = set(out["a"].ids), set(out["b"].ids)
    assert not a & b and a | b == set(range(8))
    assert {frozenset(a), frozenset(b)} == {frozenset(range(4)), frozenset(range(4, 8))}
    # node is now full: a further 1-GPU pod is infeasible there
    pod = _submit(api, "c", 1)
    ok, failed = ext.filter(pod, ["n1"])
    assert ok == [] and "insufficient" in failed["n1"]


def test_many_concurrent_binds_never_overlap():
    api, ext, _ = _cluster()
    names = [f"p{i}" for i in range(8)]
    for n in names:
        _submit(api, n, 1)
    res = {}
    errs = []

    def go(n):
        try:
            res[n] = _bind(api, ext, n)
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=go, args=(n,)) for n in names]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs
    ids = [d.ids[0] for d in res.values()]
    assert sorted(ids) == list(range(8))


def test_assume_ttl_expiry_releases_devices():
    api, ext, clock = _cluster(assume_ttl=60.0)
    _submit(api, "a", 8)
    _bind(api, ext, "a")
    _submit(api, "b", 1)
    assert ext.filter(api.get_pod("default", "b"), ["n1"])[0] == []
    clock.t += 61  # device plugin never confirmed: assumption expires (SURVEY §5.3 b)
    assert ext.filter(api.get_pod("default", "b"), ["n1"])[0] == ["n1"]


def test_confirmed_assignment_never_expires():
    api, ext, clock = _cluster(assume_ttl=60.0)
    _submit(api, "a", 8)
    _bind(api, ext, "a")
    api.patch_pod_annotations("default", "a", {ANN_ASSIGNED: "true"})  # device plugin Allocate
    clock.t += 10_000
    assert ext.filter(_submit(api, "b", 1), ["n1"])[0] == []


def test_terminal_and_deleted_pods_release():
    api, ext, _ = _cluster()
    _submit(api, "a", 8)
    _bind(api, ext, "a")
    api.set_pod_phase("default", "a", "Succeeded")
    assert ext.filter(_submit(api, "b", 8), ["n1"])[0] == ["n1"]


def test_restart_recovers_state_from_annotations():
    api, ext, clock = _cluster()
    _submit(api, "a", 4)
    d = _bind(api, ext, "a")
    ext2 = TopologyExtender(api, ExtenderConfig(resync_s=0.0), clock=clock)  # fresh process
    _submit(api, "b", 4)
    d2 = _bind(api, ext2, "b")
    assert not set(d.ids) & set(d2.ids)


def test_pods_without_group_count_as_unknown_usage():
    api, ext, _ = _cluster()
    p = api.create_pod(make_pod("legacy", gpus=6, node="n1"))  # scheduled around the extender
    ok, failed = ext.filter(_submit(api, "b", 4), ["n1"])
    assert ok == [] and "free 2" in failed["n1"]


def test_bind_failure_rolls_back_annotations():
    api, ext, _ = _cluster()
    _submit(api, "a", 2)
    api.inject("bind_pod", 500, times=1)
    with pytest.raises(Exception):
        _bind(api, ext, "a")
    ann = api.get_pod("default", "a")["metadata"]["annotations"]
    assert ANN_GROUP not in ann
    d = _bind(api, ext, "a")  # the scheduler retries: succeeds and the devices were not leaked
    assert len(d.ids) == 2


def test_transient_patch_errors_are_retried():
    api, ext, _ = _cluster()
    _submit(api, "a", 2)
    api.inject("patch_pod_annotations", 500, times=2)
    assert len(_bind(api, ext, "a").ids) == 2


def test_bind_refuses_unmanaged_pods():
    """/bind must not place pods that kube-scheduler would never delegate to the extender
    (no managed resource) or that belong to another scheduler."""
    from gpu_topology_on_k8s_amd.k8s.api import ApiError

    api, ext, _ = _cluster(scheduler_names=("default-scheduler",))
    _submit(api, "web", 0)
    with pytest.raises(ApiError) as ei:
        _bind(api, ext, "web")
    assert ei.value.code == 400 and "not managed" in str(ei.value)
    assert not api.get_pod("default", "web")["spec"].get("nodeName")
    _submit(api, "other", 2, scheduler_name="volcano")
    with pytest.raises(ApiError) as ei:
        _bind(api, ext, "other")
    assert ei.value.code == 403
    assert any(e["reason"] == "FailedGPUTopologyBind" and e["involvedObject"]["name"] == "web" for e in api.events)


def test_model_quota_gaia_b7():
    api, ext, _ = _cluster()
    c = Contract()
    pod = _submit(api, "a", 1, annotations={c.pod_model_key: "MI300X"})
    ok, failed = ext.filter(pod, ["n1"])
    assert ok == [] and "MI300X" in failed["n1"]
    pod2 = _submit(api, "b", 1, annotations={c.pod_model_key: "MI355X"})
    assert ext.filter(pod2, ["n1"])[0] == ["n1"]


def test_unhealthy_devices_excluded():
    def topo():
        t = fx.f7_mi355x()
        t.gpus[3].healthy = False
        return t

    api, ext, _ = _cluster(topo_fn=topo)
    _submit(api, "a", 7)
    d = _bind(api, ext, "a")
    assert 3 not in d.ids
    assert ext.filter(_submit(api, "b", 1), ["n1"])[0] == []


@pytest.mark.parametrize("policy", ["exact", "gaia", "design"])
def test_policies(policy):
    api, ext, _ = _cluster(policy_name=policy)
    _submit(api, "a", 4)
    d = _bind(api, ext, "a")
    assert len(set(d.ids)) == 4
    _submit(api, "b", 4)
    d2 = _bind(api, ext, "b")
    assert not set(d.ids) & set(d2.ids)


def test_gaia_policy_on_fig7_tree_node():
    """The extender with the gaia policy reproduces Table IV through the full bind path."""
    def topo():
        # Fig. 7 fixture as a topology: cost from the tree's LCA link costs
        import numpy as np

        from gpu_topology_on_k8s_amd.topology.model import GPUInfo, LinkType, Topology

        tr = fx.f4_tree()
        n = 4
        cost = np.array([[tr.pair_cost(i, j) for j in range(n)] for i in range(n)], float)
        numa = [0, 0, 1, 1]
        return Topology(gpus=[GPUInfo(index=i, numa=numa[i]) for i in range(n)],
                        link_type=np.full((n, n), int(LinkType.PCIE)), hops=np.ones((n, n), int), cost=cost)

    api, ext, _ = _cluster(topo_fn=topo, policy_name="gaia")
    api.create_pod(make_pod("x", gpus=1, node="n1", annotations=PodAssignment.assumed([2], 1_700_000_000).to_annotations()))
    _submit(api, "a", 2)
    assert _bind(api, ext, "a").ids == (0, 1)


# ------------------------------------------------------------------ HTTP wire format
def _http(ext, fn):
    async def main():
        app = make_app(ext)
        async with TestClient(TestServer(app)) as client:
            return await fn(client)

    return asyncio.run(main())


def test_http_sort_bind_filter_wire_format():
    api, ext, _ = _cluster(nodes=("n1", "n2"))
    pod = _submit(api, "p", 2)

    async def flow(client):
        r = await client.post("/gputopology-scheduler/sort", json={"Pod": pod, "NodeNames": ["n1", "n2"]})
        assert r.status == 200
        hp = await r.json()
        assert [h["Host"] for h in hp] == ["n1", "n2"] and all(0 <= h["Score"] <= 10 for h in hp)
        r = await client.post("/gputopology-scheduler/prioritize", json={"pod": pod, "nodenames": ["n1"]})
        assert (await r.json())[0]["Host"] == "n1"
        nodes = {"items": [api.get_node("n1"), api.get_node("n2")]}
        r = await client.post("/gputopology-scheduler/filter", json={"Pod": pod, "Nodes": nodes})
        fr = await r.json()
        assert [n["metadata"]["name"] for n in fr["Nodes"]["items"]] == ["n1", "n2"] and fr["Error"] == ""
        r = await client.post("/gputopology-scheduler/bind", json={"PodName": "p", "PodNamespace": "default",
                                                                     "PodUID": pod["metadata"]["uid"], "Node": "n2"})
        br = await r.json()
        assert br["Error"] == "" and len(br["Devices"]) == 2
        r = await client.post("/gputopology-scheduler/bind", json={"PodName": "p", "PodNamespace": "default",
                                                                     "PodUID": pod["metadata"]["uid"], "Node": "n2"})
        again = await r.json()  # retried bind to the same node: idempotent, same devices
        assert again["Error"] == "" and again["Devices"] == br["Devices"]
        r = await client.post("/gputopology-scheduler/bind", json={"PodName": "p", "PodNamespace": "default",
                                                                     "PodUID": pod["metadata"]["uid"], "Node": "n1"})
        assert "already bound" in (await r.json())["Error"]  # error string, HTTP 200
        r = await client.get("/gputopology-scheduler/metrics")
        text = await r.text()
        assert "gtk_extender_verb_seconds" in text and "gtk_extender_binds_total" in text
        r = await client.get("/healthz")
        assert await r.text() == "ok"
        r = await client.get("/gputopology-scheduler/debug/nodes")
        snap = await r.json()
        assert snap["n2"]["free"] == 6
        r = await client.post("/gputopology-scheduler/sort", data=b"{not json")
        assert r.status == 400

    _http(ext, flow)
    assert api.get_pod("default", "p")["spec"]["nodeName"] == "n2"


def test_prioritize_over_many_nodes_uses_constant_api_calls():
    """nodeCacheCapable: a 64-node prioritize costs one cluster-wide sync, not 2 calls per node."""
    names = tuple(f"n{i}" for i in range(64))
    api, ext, clock = _cluster(nodes=names, resync_s=5.0)
    pod = _submit(api, "p", 4)
    before = sum(api.calls.values())
    res = ext.prioritize(pod, list(names))
    used = sum(api.calls.values()) - before
    assert len(res) == 64 and all(s > 0 for _, s in res)
    assert used <= 2, dict(api.calls)
    before = sum(api.calls.values())
    ext.prioritize(pod, list(names))  # fresh cache: no API traffic at all
    assert sum(api.calls.values()) == before


def test_decision_cache_hits_and_invalidates():
    """Repeated sort calls for same-size pods on unchanged nodes are served from the LRU cache; a bind
    (new used set) misses and still yields a disjoint, correct set; random tie-breaks never cache."""
    api, ext, _ = _cluster(nodes=("n1", "n2"))
    p1, p2 = _submit(api, "a", 4), _submit(api, "b", 4)
    first = ext.prioritize(p1, ["n1", "n2"])
    assert ext.prioritize(p2, ["n1", "n2"]) == first
    assert ext.metrics.decision_cache.labels(result="hit")._value.get() >= 2
    d1 = _bind(api, ext, "a")  # bind re-evaluates: cached decision for (n1, {}, 4)
    d2 = _bind(api, ext, "b")  # used set changed -> miss -> the other half
    assert not set(d1.ids) & set(d2.ids)
    p3 = _submit(api, "c", 4)
    cached = ext.prioritize(p3, ["n1", "n2"])
    ext.cfg.decision_cache = 0  # same extender state, cache off: same answer
    assert cached == ext.prioritize(p3, ["n1", "n2"]) and cached[0][1] == 0  # n1 is full now

    from gpu_topology_on_k8s_amd.placement import PlacementPolicy

    _, rnd, _ = _cluster(policy=PlacementPolicy(tie_break="random"))
    assert not rnd._cacheable()


def test_node_memo_tracks_state_version_and_assumption_expiry():
    """The per-node memo answers a same-shape pod without re-evaluating; any usage change (bind,
    watch event) or the expiry of a live assumption invalidates it, and pod shapes never mix."""
    api, ext, clock = _cluster(assume_ttl=60.0)
    st = ext.cache.get("n1")
    a = _submit(api, "a", 4)
    ext.prioritize(a, ["n1"])
    v0, memo0 = st.version, dict(st.memo)
    assert len(memo0) == 1
    ext.prioritize(_submit(api, "a2", 4), ["n1"])
    assert st.version == v0 and st.memo == memo0  # served from the memo
    ext.prioritize(_submit(api, "pinned", 4, annotations={Contract().numa_pref_key: "1"}), ["n1"])
    assert len(st.memo) == 2  # a NUMA preference is another shape
    _bind(api, ext, "a")
    assert st.version > v0
    b = _submit(api, "b", 4)
    ok, _ = ext.filter(b, ["n1"])
    assert ok == ["n1"]
    _submit(api, "c", 1)
    assert ext.filter(api.get_pod("default", "c"), ["n1"])[0] == ["n1"]
    _submit(api, "big", 8)
    assert ext.filter(api.get_pod("default", "big"), ["n1"])[0] == []  # 4 assumed
    clock.t += 61  # the assumption of "a" expires without any state change
    assert ext.filter(api.get_pod("default", "big"), ["n1"])[0] == ["n1"]
    v1 = st.version
    ext.cache.on_event("MODIFIED", "Pod", api.get_pod("default", "a"))
    assert st.version > v1 and not st.memo


def _running(api, ext, name, k):
    """A bound, Allocate-confirmed pod holding k devices."""
    pod = _submit(api, name, k)
    d = ext.bind("default", name, pod["metadata"]["uid"], "n1")
    api.patch_pod_annotations("default", name, {ANN_ASSIGNED: "true"})
    return api.get_pod("default", name), d


def test_preempt_keeps_the_smallest_victim_set_with_the_best_topology():
    """kube-scheduler proposes every lower-priority pod; a 4-GPU pod needs only the two 2-GPU pods of
    one NUMA half gone.  The extender keeps those two, drops the rest, and keeps non-GPU victims."""
    api, ext, _ = _cluster()
    held = [_running(api, ext, f"p{i}", 2) for i in range(4)]  # 0-1, 2-3 | 4-5, 6-7 (or similar)
    uids = [p["metadata"]["uid"] for p, _ in held]
    cpu_only = api.create_pod(make_pod("cpu-only", gpus=0))["metadata"]["uid"]
    pod = _submit(api, "big", 4)
    res = ext.preempt(pod, {"n1": (uids + [cpu_only], 1)})
    kept, pdb = res["n1"]
    assert pdb == 1 and cpu_only in kept
    gpu_kept = [u for u in kept if u != cpu_only]
    assert len(gpu_kept) == 2
    freed = set()
    for (p, d) in held:
        if p["metadata"]["uid"] in gpu_kept:
            freed |= set(d.ids)
    numa = {fx.f7_mi355x().gpus[i].numa for i in freed}
    assert len(freed) == 4 and len(numa) == 1  # a whole NUMA half, not one pair from each side


def test_preempt_drops_nodes_where_victims_do_not_suffice():
    api, ext, _ = _cluster()
    held = [_running(api, ext, f"q{i}", 4) for i in range(2)]
    pod = _submit(api, "all8", 8)
    one = held[0][0]["metadata"]["uid"]
    assert ext.preempt(pod, {"n1": ([one], 0)}) == {}
    both = [p["metadata"]["uid"] for p, _ in held]
    assert sorted(ext.preempt(pod, {"n1": (both, 0)})["n1"][0]) == sorted(both)
    # a node under a re-probe mark offers no preemption either (deviceplugin/plugin.py reprobe)
    api.patch_node("n1", annotations={Contract().probing_key: str(int(time.time()) + 300)})
    ext.cache.refresh_node("n1")
    assert ext.preempt(pod, {"n1": (both, 0)}) == {}


def test_http_preempt_wire_format():
    api, ext, _ = _cluster()
    held = [_running(api, ext, f"w{i}", 4) for i in range(2)]
    pod = _submit(api, "want4", 4)
    args = {"Pod": pod, "NodeNameToMetaVictims": {"n1": {"Pods": [{"UID": p["metadata"]["uid"]} for p, _ in held],
                                                          "NumPDBViolations": 0}}}

    async def go():
        async with TestClient(TestServer(make_app(ext))) as client:
            r = await client.post("/gputopology-scheduler/preempt", json=args)
            return r.status, await r.json()

    status, body = asyncio.run(go())
    assert status == 200
    pods = body["NodeNameToMetaVictims"]["n1"]["Pods"]
    assert len(pods) == 1 and body["NodeNameToMetaVictims"]["n1"]["NumPDBViolations"] == 0


def test_multi_node_pod_binds_across_nic_domains():
    def topo():
        t = fx.f7_mi355x()
        t.nics = [{"name": "mlx5_0", "state": "4: ACTIVE"}, {"name": "mlx5_1", "state": "4: ACTIVE"}]
        t.gpu_nic = [[1, 5] if i < 4 else [5, 1] for i in range(8)]
        return t

    api, ext, _ = _cluster(topo_fn=topo)
    _submit(api, "mn", 2, annotations={Contract().multi_node_key: "true"})
    d = _bind(api, ext, "mn")
    assert {i // 4 for i in d.ids} == {0, 1}
    _submit(api, "local", 2)
    d2 = _bind(api, ext, "local")
    assert len({i // 4 for i in d2.ids}) == 1
    rdma = api.create_pod(make_pod("rdma", gpus=2))
    rdma["spec"]["containers"][0]["resources"]["limits"]["rdma/hca"] = "1"
    assert ext.multi_node(rdma) and not ext.multi_node(api.get_pod("default", "local"))


def test_a_pod_with_a_garbage_group_annotation_does_not_break_its_node():
    """Any user can annotate their own pod: a GROUP that is not a device list must not stop the
    extender from reading the node (the pod counts by its request, like a pod without a GROUP)."""
    api, ext, _ = _cluster()
    for i, bad in enumerate(("x,1", "-1", "1,,2,a", "0x1")):
        api.create_pod(make_pod(f"odd{i}", gpus=1, node="n1", annotations={ANN_GROUP: bad, ANN_ASSIGNED: "true"}))
    assert PodAssignment.from_annotations({ANN_GROUP: "x,1"}) is None
    assert PodAssignment.from_annotations({ANN_GROUP: "1,,2"}).group == [1, 2]  # empty entries are skipped
    _submit(api, "p", 4)
    d = _bind(api, ext, "p")
    assert d is not None and len(d.ids) == 4
    _submit(api, "big", 8)
    with pytest.raises(Exception):
        _bind(api, ext, "big", "n1")  # 4 (p) + 3 unreadable-but-counted + "1,,2" holding 1,2: no room for 8
