"""Nodes whose kubelet runs the Topology Manager (placement/numa_align.py).

The kubelet offers each container the free devices of the narrowest, lowest NUMA set that fits, and a
``restricted`` or ``single-numa-node`` kubelet rejects pods that do not align (``TopologyAffinityError``,
pod Failed for good).  The extender replays that procedure, so the GROUP it binds is what the kubelet
allocates, and it never binds a pod the kubelet would reject.  The fake kubelet
(deviceplugin/kubelet.py) implements the Topology Manager separately, in the kubelet's own structure
(bitmask hints, ``mergeFilteredHints``, ``filterByAffinity``); these tests hold the two against each
other."""
import random

import pytest

from gpu_topology_on_k8s_amd.deviceplugin.__main__ import topology_manager_of
from gpu_topology_on_k8s_amd.k8s import Contract, PodAssignment
from gpu_topology_on_k8s_amd.k8s.objects import annotations as obj_annotations
from gpu_topology_on_k8s_amd.k8s.objects import labels as obj_labels
from gpu_topology_on_k8s_amd.placement.numa_align import (TopologyManager, best_hint, plan, read_kubelet_config,
                                                          tm_from_labels)
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx

NUMA = {i: 0 if i < 4 else 1 for i in range(8)}  # F7: GPUs 0-3 on NUMA node 0, 4-7 on node 1
ALL = list(range(8))


def _hint(policy, k, used, reusable=()):
    return best_hint(policy, k, set(ALL) - set(used) - set(reusable), set(reusable), NUMA, ALL)


@pytest.mark.parametrize("policy", ["best-effort", "restricted", "single-numa-node"])
def test_hints_pick_the_lowest_numa_node_that_fits(policy):
    assert _hint(policy, 2, []) == (frozenset({0}), True, True)
    assert _hint(policy, 2, [0, 1, 2]) == (frozenset({1}), True, True)
    assert _hint(policy, 4, [5]) == (frozenset({0}), True, True)


def test_a_request_no_numa_node_holds_any_more_is_not_preferred():
    used = [0, 1, 2, 4, 5, 6]  # one free GPU per NUMA node: a 2-GPU pod could sit on one node of an empty machine
    assert _hint("best-effort", 2, used) == (frozenset({0, 1}), False, True)
    assert _hint("restricted", 2, used)[2] is False
    assert _hint("single-numa-node", 2, used) == (None, False, False)


def test_a_request_wider_than_a_numa_node():
    assert _hint("restricted", 6, []) == (frozenset({0, 1}), True, True)  # minimal width is 2: preferred
    assert _hint("single-numa-node", 6, [])[2] is False


def test_reused_devices_pin_the_hint():
    # an init container's devices on NUMA node 1 are handed on: only masks holding them qualify
    assert _hint("best-effort", 2, [], reusable=[4]) == (frozenset({1}), True, True)
    assert _hint("single-numa-node", 2, [5, 6, 7], reusable=[4, 0])[2] is False


def _first(n, offered, must):
    out = sorted(must)
    return out + [d for d in sorted(offered) if d not in out][: n - len(out)]


def test_plan_follows_the_device_managers_two_branches():
    t = fx.f7_mi355x()
    tm = TopologyManager("best-effort", "container")
    # needed < aligned: the plugin chooses among NUMA node 0's free devices only
    assert plan(t, [0], [(2, "app")], tm, lambda n, off, must: sorted(off, reverse=True)[:n]) == ((2, 3), "")
    # needed == aligned: every aligned device, no choice left
    assert plan(t, [0], [(3, "app")], tm, _first) == ((1, 2, 3), "")
    # needed > aligned (6 devices, minimal width 2): everything is aligned
    assert plan(t, [], [(6, "app")], tm, _first) == ((0, 1, 2, 3, 4, 5), "")
    # per container: the second container finds NUMA node 0 too full and goes to node 1
    assert plan(t, [0], [(2, "app"), (2, "app")], tm, _first) == ((1, 2, 4, 5), "")
    # scope pod: one hint for the pod's 4 devices, both containers inside it
    assert plan(t, [0], [(2, "app"), (2, "app")], TopologyManager("best-effort", "pod"), _first) == ((4, 5, 6, 7), "")
    ids, why = plan(t, [], [(6, "app")], TopologyManager("single-numa-node", "container"), _first)
    assert ids is None and "TopologyAffinityError" in why


def _shape(rng):
    """A random pod: one or two app containers, sometimes an init container, 1..8 GPUs in total."""
    r = rng.random()
    if r < 0.5:
        return {"gpus": rng.choice([1, 1, 2, 2, 3, 4, 6, 8])}
    if r < 0.8:
        a, b = rng.choice([(1, 1), (1, 2), (2, 2), (1, 3), (2, 4)])
        return {"gpus": 0, "split": [a, b]}
    app = rng.choice([1, 2, 3])
    return {"gpus": 0, "split": [app], "init": [rng.choice([1, 2, app])]}


@pytest.mark.parametrize("policy,scope,split,n", [("best-effort", "container", 2, 8), ("restricted", "container", 2, 8),
                                                  ("single-numa-node", "container", 2, 8), ("best-effort", "pod", 2, 8),
                                                  ("single-numa-node", "pod", 2, 8), ("best-effort", "container", 4, 8),
                                                  ("restricted", "pod", 4, 8), ("best-effort", "container", 4, 16),
                                                  ("restricted", "container", 4, 16)])
def test_groups_equal_what_the_kubelet_allocates_under_churn(policy, scope, split, n):
    """Random pods arrive and finish on two MI355X nodes whose kubelets run the Topology Manager (hosts
    with 2 NUMA nodes, or 4 as an EPYC in NPS2/NPS4 mode; 16 devices are a node of DPX partitions, 4 per
    NUMA node); the reconcile pass is off.  Every pod the extender binds
    is admitted with exactly its GROUP, and no pod is bound that the kubelet rejects."""
    from gpu_topology_on_k8s_amd.topology.model import Topology

    rng = random.Random(f"{policy}/{scope}/{split}/{n}")
    tm = TopologyManager(policy, scope)
    node = lambda: Topology.full_mesh(n=n, numa_split=split, node_name="mi355x")  # noqa: E731
    with SimCluster({"a": node(), "b": node()}, topology_manager=tm) as c:
        live = []
        placed = 0
        for i in range(40):
            if live and rng.random() < 0.4:
                c.complete(live.pop(rng.randrange(len(live))))
            c.submit(f"p{i}", **_shape(rng))
            (r,) = c.schedule_pending()
            if r.node is None:
                assert r.error, r
                c.delete(f"p{i}")  # infeasible now: a real scheduler would retry it later
                continue
            assert not r.error, r  # bound means admitted: the kubelet rejected nothing the extender bound
            # what the extender decided at bind is what the kubelet allocated (the plugin did not have to
            # correct the GROUP at Allocate), and the annotation says so
            assert sorted(r.devices) == sorted(r.allocated), (i, r)
            pa = PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", f"p{i}")))
            assert sorted(pa.group) == sorted(r.allocated) and pa.assigned, (i, pa, r)
            live.append(f"p{i}")
            placed += 1
        assert placed >= 15
        assert not any(rej for n in c.nodes.values() for rej in n.kubelet.rejected)
        assert sum(n.plugin.metrics.group_overridden._value.get() for n in c.nodes.values()) == 0


def test_an_untold_plugin_shows_the_kubelet_overriding_groups():
    """The operator did not tell the plugin the kubelet's ``best-effort`` policy: the extender binds
    devices the kubelet does not offer, the plugin records what the kubelet chose, and
    ``gtk_plugin_group_overridden_total`` says so (docs/OPERATIONS.md)."""
    rng = random.Random("best-effort/container/2")
    tm = TopologyManager("best-effort", "container")
    with SimCluster({"a": fx.f7_mi355x(), "b": fx.f7_mi355x()}, topology_manager=tm, publish_topology_manager=False) as c:
        live, differ = [], 0
        for i in range(40):
            if live and rng.random() < 0.4:
                c.complete(live.pop(rng.randrange(len(live))))
            c.submit(f"p{i}", **_shape(rng))
            (r,) = c.schedule_pending()
            if r.node is None or r.error:
                c.delete(f"p{i}")
                continue
            differ += sorted(r.devices) != sorted(r.allocated)
            live.append(f"p{i}")
        overridden = sum(n.plugin.metrics.group_overridden._value.get() for n in c.nodes.values())
        text = "".join(n.plugin.metrics.exposition().decode() for n in c.nodes.values())
    assert differ > 0 and overridden >= differ
    assert "gtk_plugin_group_overridden_total" in text


def test_an_extender_that_ignores_the_policy_loses_pods_the_aware_one_places():
    """``single-numa-node`` kubelets, two nodes with room for 4 GPUs each, but only node b has them on
    one NUMA node.  Unaware, the extender binds to node a, where the kubelet rejects the pod for good
    (Failed, TopologyAffinityError); aware, it filters node a out with the reason and places the pod on b."""
    tm = TopologyManager("single-numa-node", "container")
    results = {}
    for aware in (False, True):
        with SimCluster({"a": fx.f7_mi355x(), "b": fx.f7_mi355x()}, topology_manager=tm,
                        publish_topology_manager=aware) as c:
            # node a: 2 GPUs used on each NUMA node (four 2-GPU pods, two of them done); node b: NUMA node 0 full
            for node, groups, done in (("a", ([0, 1], [2, 3], [4, 5], [6, 7]), (1, 3)), ("b", ([0, 1], [2, 3]), ())):
                for j, g in enumerate(groups):
                    name = f"pre-{node}{j}"
                    c.submit(name, 2)
                    uid = c.api.get_pod("default", name)["metadata"]["uid"]
                    c.api.patch_pod_annotations("default", name, PodAssignment(g, False, 0).to_annotations())
                    c.api.bind_pod("default", name, uid, node)
                    c.nodes[node].kubelet.admit(c.api.get_pod("default", name), c.resource)
                    assert sorted(int(d) for d in c.nodes[node].kubelet.allocated[c.resource][f"default/{name}"]) == g
                for j in done:
                    c.complete(f"pre-{node}{j}")
            c.extender.cache.sync_all()
            c.submit("x", 4)
            fr = c.extender.filter(c.api.get_pod("default", "x"), ["a", "b"])
            (r,) = c.schedule_pending()
            results[aware] = (r, fr, c.api.get_pod("default", "x"))
    r, fr, pod = results[True]
    assert r.node == "b" and not r.error and sorted(r.allocated) == [4, 5, 6, 7]
    assert "TopologyAffinityError" in fr[1]["a"]
    r, _, pod = results[False]  # both nodes score 10 on links alone; the tie goes to a, and the pod is lost
    assert r.node == "a" and "TopologyAffinityError" in r.error and pod["status"]["phase"] == "Failed"


def test_the_plugin_publishes_the_policy_from_flags_or_the_kubelet_config(tmp_path):
    cfgfile = tmp_path / "config.yaml"
    cfgfile.write_text("apiVersion: kubelet.config.k8s.io/v1beta1\nkind: KubeletConfiguration\n"
                       "topologyManagerPolicy: single-numa-node\ntopologyManagerScope: pod\n")
    assert read_kubelet_config(str(cfgfile)) == TopologyManager("single-numa-node", "pod")

    class A:
        topology_manager_policy = ""
        topology_manager_scope = ""
        kubelet_config = str(cfgfile)

    assert topology_manager_of(A) == TopologyManager("single-numa-node", "pod")
    A.topology_manager_policy = "restricted"
    assert topology_manager_of(A) == TopologyManager("restricted", "pod")  # a flag beats the file
    A.kubelet_config = str(tmp_path / "missing.yaml")
    A.topology_manager_policy = ""
    assert topology_manager_of(A) == TopologyManager()
    with SimCluster({"a": fx.f7_mi355x()}, topology_manager=TopologyManager("restricted", "container")) as c:
        labels = obj_labels(c.api.get_node("a"))
        assert tm_from_labels(labels, Contract().prefix) == TopologyManager("restricted", "container")
    assert tm_from_labels({f"{Contract().prefix}/topology-manager-policy": "bogus"}, Contract().prefix) == TopologyManager()


def test_the_manifests_hand_the_policy_to_the_plugin():
    import yaml

    from gpu_topology_on_k8s_amd.config import render_manifests

    def plugin_cmd(**kw):
        docs = list(yaml.safe_load_all(render_manifests(**kw)))
        ds = next(d for d in docs if d["kind"] == "DaemonSet" and "device-plugin" in d["metadata"]["name"])
        return ds["spec"]["template"]["spec"]["containers"][0]["command"]

    assert not any("topology-manager" in a for a in plugin_cmd())
    cmd = plugin_cmd(topology_manager_policy="single-numa-node", topology_manager_scope="pod")
    assert "--topology-manager-policy=single-numa-node" in cmd and "--topology-manager-scope=pod" in cmd


def test_init_container_devices_are_reused_under_the_topology_manager():
    """An init container's devices go on to the app container (the kubelet's devicesToReuse), also
    when its hint is computed: the pod holds max(init, app) devices, never their sum."""
    t = fx.f7_mi355x()
    tm = TopologyManager("single-numa-node", "container")
    assert plan(t, [], [(2, "init"), (2, "app")], tm, _first) == ((0, 1), "")
    assert plan(t, [], [(1, "init"), (3, "app")], tm, _first) == ((0, 1, 2), "")
    assert plan(t, [0, 1], [(1, "sidecar"), (2, "app")], tm, _first) == ((2, 4, 5), "")  # a sidecar keeps its GPU
    with SimCluster({"a": fx.f7_mi355x()}, topology_manager=tm) as c:
        c.submit("warm", 0, split=[3], init=[2])
        c.submit("side", 0, split=[2], sidecars=[1])
        for r in c.schedule_pending():
            assert r.node == "a" and not r.error and sorted(r.devices) == sorted(r.allocated), r
        assert [sorted(r.allocated) for r in c.history] == [[0, 1, 2], [3, 4, 5]]


def test_preemption_counts_only_victims_whose_devices_the_kubelet_would_align():
    """Victims that free one GPU on each NUMA node make room for a 2-GPU pod by count, but a
    ``single-numa-node`` kubelet would reject it there: /preempt drops the node."""
    import time

    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
    from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
    from gpu_topology_on_k8s_amd.placement.numa_align import tm_labels

    c = Contract()
    for tm, expect in ((TopologyManager(), True), (TopologyManager("single-numa-node", "container"), False)):
        api = FakeAPIServer()
        api.create_node(make_node("n1", labels=tm_labels(tm, c.prefix), annotations=encode_node_annotations(fx.f7_mi355x(), c),
                                  capacity={c.resource_name: "8"}))
        uids = {}
        for name, ids in (("a", [0]), ("b", [4]), ("c", [1, 2, 3]), ("d", [5, 6, 7])):
            p = api.create_pod(make_pod(name, gpus=len(ids), node="n1",
                                        annotations=PodAssignment(ids, True, int(time.time())).to_annotations()))
            uids[name] = p["metadata"]["uid"]
        ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
        pod = api.create_pod(make_pod("want2", gpus=2))
        got = ext.preempt(pod, {"n1": ([uids["a"], uids["b"]], 0)})
        assert ("n1" in got) is expect, (tm, got)


@pytest.mark.parametrize("split", [2, 4, 8])
def test_the_extenders_hints_equal_the_fake_kubelets(split):
    """Differential check of the two implementations (placement/numa_align.best_hint against the fake
    kubelet's bitmask hints and merge) over random states, on hosts with 2, 4 and 8 NUMA nodes (an EPYC
    host in NPS4 mode puts one MI355X on each): same admission, same hinted NUMA nodes."""
    from gpu_topology_on_k8s_amd.deviceplugin.kubelet import FakeKubelet, _bits, _Plugin
    from gpu_topology_on_k8s_amd.topology.model import Topology

    t = Topology.full_mesh(n=8, numa_split=split)
    numa = {g.index: int(g.numa) for g in t.gpus}
    assert len(set(numa.values())) == split
    rng = random.Random(split)
    for policy in ("best-effort", "restricted", "single-numa-node"):
        kl = FakeKubelet("/nonexistent", topology_policy=policy)
        p = _Plugin(resource="amd.com/gpu", endpoint="", channel=None, options=None,
                    devices={str(i): "Healthy" for i in range(8)}, numa={str(i): (numa[i],) for i in range(8)})
        for _ in range(300):
            used = set(rng.sample(range(8), rng.randint(0, 7)))
            reusable = set(rng.sample(sorted(used), rng.randint(0, min(2, len(used)))))  # the pod's own init devices
            avail = set(range(8)) - used
            req = rng.randint(1, 8)
            mask, admit = kl._merge(p, kl._generate_hints(p, {str(d) for d in avail}, {str(d) for d in reusable}, req))
            want, _, ok = best_hint(policy, req, avail, reusable, numa, list(range(8)))
            assert ok == admit, (policy, used, reusable, req)
            assert (None if mask is None else frozenset(_bits(mask))) == want, (policy, used, reusable, req)


def test_equally_narrow_hints_tie_break_on_the_bitmask_value():
    """16 devices, 4 per NUMA node on 4 nodes; free counts 1, 3, 2, 4 and a request of 5: both {0,3} and
    {1,2} hold it, neither {0,1} nor {0,2} does.  The kubelet's IsNarrowerThan compares equal-width
    masks as integers (0b0110 < 0b1001), so it hints {1,2}, not the lexicographically first {0,3}; the
    extender and the fake kubelet agree with it."""
    from gpu_topology_on_k8s_amd.deviceplugin.kubelet import FakeKubelet, _bits, _Plugin

    numa = {d: d // 4 for d in range(16)}
    free = {0} | {4, 5, 6} | {8, 9} | {12, 13, 14, 15}
    for policy in ("best-effort", "restricted"):
        assert best_hint(policy, 5, free, set(), numa, list(range(16))) == (frozenset({1, 2}), True, True)
        kl = FakeKubelet("/nonexistent", topology_policy=policy)
        p = _Plugin(resource="amd.com/gpu", endpoint="", channel=None, options=None,
                    devices={str(i): "Healthy" for i in range(16)}, numa={str(i): (numa[i],) for i in range(16)})
        mask, admit = kl._merge(p, kl._generate_hints(p, {str(d) for d in free}, set(), 5))
        assert admit and set(_bits(mask)) == {1, 2}


def test_the_hints_agree_on_sixteen_devices_over_four_numa_nodes():
    """The differential check on 4 devices per NUMA node, where equal-width ties between masks are
    common."""
    from gpu_topology_on_k8s_amd.deviceplugin.kubelet import FakeKubelet, _bits, _Plugin

    numa = {d: d // 4 for d in range(16)}
    rng = random.Random(16)
    for policy in ("best-effort", "restricted", "single-numa-node"):
        kl = FakeKubelet("/nonexistent", topology_policy=policy)
        p = _Plugin(resource="amd.com/gpu", endpoint="", channel=None, options=None,
                    devices={str(i): "Healthy" for i in range(16)}, numa={str(i): (numa[i],) for i in range(16)})
        for _ in range(300):
            used = set(rng.sample(range(16), rng.randint(0, 15)))
            reusable = set(rng.sample(sorted(used), rng.randint(0, min(3, len(used)))))
            avail = set(range(16)) - used
            req = rng.randint(1, 12)
            mask, admit = kl._merge(p, kl._generate_hints(p, {str(d) for d in avail}, {str(d) for d in reusable}, req))
            want, _, ok = best_hint(policy, req, avail, reusable, numa, list(range(16)))
            assert ok == admit and (None if mask is None else frozenset(_bits(mask))) == want, (policy, used, reusable, req)


@pytest.mark.gpu
def test_a_real_node_under_single_numa_node():
    """The MI355X of the box, discovered through amdsmi with the NUMA node its host reports (not
    necessarily 0), advertised as 4 time slices, its kubelet under ``single-numa-node``: the devices'
    TopologyInfo carries that NUMA node, every pod is admitted with exactly the GROUP the extender
    bound, and the node labels name the policy."""
    from gpu_topology_on_k8s_amd.topology.discovery import discover
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    t = discover("auto")
    t.node_name = "gpu-node"
    v = time_slice(t, 4)
    numa = {int(g.numa) for g in v.gpus}
    tm = TopologyManager("single-numa-node", "container")
    with SimCluster({"gpu-node": v}, topology_manager=tm, reconcile_interval=0.0) as c:
        kub = c.nodes["gpu-node"].kubelet
        res = c.nodes["gpu-node"].resource
        assert {n for ns in kub.plugins[res].numa.values() for n in ns} == numa
        assert tm_from_labels(obj_labels(c.api.get_node("gpu-node")), Contract().prefix) == tm
        c.submit("two", 0, split=[1, 1], slices=True)
        c.submit("pair", 2, slices=True)
        for r in c.schedule_pending():
            assert not r.error and sorted(r.devices) == sorted(r.allocated), r
        assert not kub.rejected
    print({"numa_nodes": sorted(numa), "devices": v.n})


def test_doctor_names_the_plugin_flags_the_kubelet_needs(tmp_path):
    from gpu_topology_on_k8s_amd.doctor import check_topology_manager

    assert check_topology_manager(str(tmp_path / "none.yaml"))["status"] == "skip"
    f = tmp_path / "config.yaml"
    f.write_text("kind: KubeletConfiguration\ntopologyManagerPolicy: restricted\n")
    c = check_topology_manager(str(f))
    assert c["status"] == "ok" and c["policy"] == "restricted" and "--topology-manager-policy=restricted" in c["detail"]
    f.write_text("kind: KubeletConfiguration\ntopologyManagerPolicy: bogus\n")
    assert check_topology_manager(str(f))["status"] == "fail"
    # policy options: prefer-closest-numa-nodes changes the hint tie-break the extender replays -> warned
    f.write_text("kind: KubeletConfiguration\ntopologyManagerPolicy: best-effort\n"
                 "topologyManagerPolicyOptions:\n  prefer-closest-numa-nodes: \"true\"\n  max-allowable-numa-nodes: \"16\"\n")
    c = check_topology_manager(str(f))
    assert c["status"] == "warn" and c["options"] == ["prefer-closest-numa-nodes"] and "overridden" in c["detail"]
    f.write_text("kind: KubeletConfiguration\ntopologyManagerPolicy: best-effort\n"
                 "topologyManagerPolicyOptions:\n  prefer-closest-numa-nodes: \"false\"\n  max-allowable-numa-nodes: \"16\"\n")
    assert check_topology_manager(str(f))["status"] == "ok"


@pytest.mark.parametrize("used,reusable,size,want", [
    ((), (), 1, [({0}, True), ({1}, True), ({0, 1}, False)]),
    ((), (), 2, [({0}, True), ({1}, True), ({0, 1}, False)]),
    ((), (), 3, [({0, 1}, True)]),
    (("2", "3"), (), 2, [({0, 1}, False)]),  # one free GPU per NUMA node: no narrow hint left, none preferred
    (("1", "3"), (), 2, [({0}, True), ({0, 1}, False)]),  # node 1 full: node 0 still holds the pair
    (("3",), ("3",), 2, [({1}, True), ({0, 1}, False)]),  # a reused GPU on node 1 pins every mask to contain 1
    (("0", "1", "2", "3"), (), 1, []),  # nothing free: no hint at all
])
def test_the_fake_kubelets_hint_lists(used, reusable, size, want):
    """The device manager's hints for 4 GPUs, two per NUMA node (``generateDeviceTopologyHints``): every
    NUMA set whose free plus reused devices hold the request, preferred when as narrow as the narrowest
    set whose devices, free or not, could."""
    from gpu_topology_on_k8s_amd.deviceplugin.kubelet import FakeKubelet, _bits, _Plugin

    kl = FakeKubelet("/nonexistent", topology_policy="best-effort")
    p = _Plugin(resource="amd.com/gpu", endpoint="", channel=None, options=None, devices={str(i): "Healthy" for i in range(4)},
                numa={"0": (0,), "1": (1,), "2": (0,), "3": (1,)})
    avail = {str(i) for i in range(4)} - set(used)
    hints = kl._generate_hints(p, avail - set(reusable), set(reusable), size)
    assert [(set(_bits(m)), pref) for m, pref in hints] == want


def test_an_allocation_without_preferred_call_after_a_finished_pod_is_a_new_pod():
    """Under a Topology Manager the kubelet skips GetPreferredAllocation when the aligned devices are
    exactly what a container needs, so "no preferred call" does not mean "reused devices".  Pod p1 has
    ended on the kubelet (its GPUs freed) while the apiserver still shows it Running; p2 gets p1's GPUs
    with no preferred call.  The plugin must not take that call for p1 (whose admission finished): p2
    is claimed, with the devices the kubelet gave it."""
    tm = TopologyManager("best-effort", "container")
    with SimCluster({"n": fx.f7_mi355x()}, topology_manager=tm) as c:
        kub, res = c.nodes["n"].kubelet, c.resource
        c.submit("p0", 2)
        c.submit("p1", 2)
        r0, r1 = c.schedule_pending()
        assert sorted(r0.allocated) == [0, 1] and sorted(r1.allocated) == [2, 3]
        n_pref = len(kub.preferred_calls)
        kub.release(c.api.get_pod("default", "p1"))  # the kubelet freed p1's GPUs; its status update lags
        c.submit("p2", 2)
        (r2,) = c.schedule_pending()
        assert sorted(r2.allocated) == [2, 3] and len(kub.preferred_calls) == n_pref  # aligned == needed: no preferred call
        pa2 = PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", "p2")))
        pa1 = PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", "p1")))
        assert pa2.assigned and sorted(pa2.group) == [2, 3], pa2
        assert sorted(pa1.group) == [2, 3] and pa1.assigned
