"""Multi-container and init-container GPU pods through the real per-container kubelet protocol
(reference ``design.md:236-246``).

The kubelet's device manager calls ``GetPreferredAllocation`` and ``Allocate`` once per container with
that container's count; a regular init container's devices are reused by the containers after it.
The extender's GROUP covers the whole pod, so the plugin must hand out GROUP sub-parts and flip
``ASSIGNED=true`` once the GROUP is fully claimed.  Every test here runs with the pod-resources
reconcile pass disabled (``SimCluster`` default ``reconcile_interval=0`` and ``reconcile()`` never
called before the assertions): the Allocate path alone must get it right.
"""
import pytest

from gpu_topology_on_k8s_amd.deviceplugin import proto as pb
from gpu_topology_on_k8s_amd.k8s import Contract, PodAssignment
from gpu_topology_on_k8s_amd.k8s.objects import annotations as obj_annotations
from gpu_topology_on_k8s_amd.k8s.objects import make_pod, pod_device_steps, pod_gpu_request
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx

RES = "amd.com/gpu"


def _ann(c, name):
    return PodAssignment.from_annotations(obj_annotations(c.api.get_pod("default", name)))


def _busy_node(c):
    """A partially used 8-GPU node: a 1-GPU and a 2-GPU pod already run there."""
    c.submit("busy1", 1)
    c.submit("busy2", 2)
    rs = c.schedule_pending()
    assert all(r.allocated for r in rs)
    return {i for r in rs for i in r.allocated}


def _calls(kub, name):
    return [(cname, tuple(sorted(int(i) for i in ids))) for key, cname, ids in kub.allocate_calls if key == f"default/{name}"]


@pytest.mark.parametrize("shape", [
    dict(split=[2, 2]),
    dict(split=[1, 3]),
    dict(split=[2, 0, 2]),  # a container without devices in between: no call for it
    dict(split=[1, 1, 1, 1]),
])
def test_app_containers_each_get_a_part_of_the_group(shape):
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        busy = _busy_node(c)
        c.submit("mc", 0, **shape, annotations={f"{Contract().prefix}/rccl-env": "NCCL_MIN_NCHANNELS=16"})
        (r,) = c.schedule_pending()
        kub = c.nodes["n"].kubelet
        group = sorted(r.devices)
        assert len(group) == sum(shape["split"]) and not set(group) & busy
        pa = _ann(c, "mc")
        assert pa.assigned and sorted(pa.group) == group  # exactly the extender's GROUP, no reconcile
        assert sorted(int(i) for i in kub.allocated[RES]["default/mc"]) == group
        calls = _calls(kub, "mc")
        assert [len(ids) for _, ids in calls] == [n for n in shape["split"] if n]  # one Allocate per container
        seen = [i for _, ids in calls for i in ids]
        assert sorted(seen) == group  # disjoint parts covering the GROUP
        for cr in kub.responses["default/mc"].container_responses:
            assert cr.envs["NCCL_MIN_NCHANNELS"] == "16"  # every container keeps the pod's rccl-env
        assert c.used_devices("n") == sorted(busy | set(group))


@pytest.mark.parametrize("split,init,group", [
    ([2, 2], [], [1, 3, 4, 6]),
    ([1, 3], [], [0, 2, 5, 7]),
    ([4], [2], [1, 2, 5, 6]),
    ([2], [4], [0, 3, 4, 7]),
])
def test_an_arbitrary_group_is_followed_exactly(split, init, group):
    """A GROUP the placement core would never pick by itself (spread over both NUMA halves): the
    containers get exactly it, so the answers come from the annotation, not from a placement rerun."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        pod = c.api.create_pod(make_pod("arb", split=split, init=init, node="n",
                                        annotations=PodAssignment.assumed(group, 1).to_annotations()))
        kub = c.nodes["n"].kubelet
        kub.admit(pod, c.resource)
        assert sorted(int(i) for i in kub.allocated[RES]["default/arb"]) == group
        pa = _ann(c, "arb")
        assert pa.assigned and sorted(pa.group) == group
        for _, ids in _calls(kub, "arb"):
            assert set(ids) <= set(group)


def test_init_then_larger_app_container_reuses_the_init_devices():
    """init(2) + app(4): the init container gets 2 of the GROUP; the app container gets those 2 back
    (must_include) plus the other 2 through GetPreferredAllocation."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        busy = _busy_node(c)
        c.submit("ia", 0, split=[4], init=[2])
        (r,) = c.schedule_pending()
        kub = c.nodes["n"].kubelet
        group = sorted(r.devices)
        assert len(group) == 4 and not set(group) & busy
        (ic, init_ids), (ac, app_ids) = _calls(kub, "ia")
        assert ic == "init0" and ac == "c0"
        assert set(init_ids) < set(group) and app_ids == tuple(group)
        must, size = kub.preferred_calls[-1]
        assert sorted(int(i) for i in must) == sorted(init_ids) and size == 4
        pa = _ann(c, "ia")
        assert pa.assigned and sorted(pa.group) == group
        assert c.used_devices("n") == sorted(busy | set(group))


def test_init_larger_than_app_keeps_the_whole_group():
    """init(4) + app(2): the init container claims the whole GROUP (ASSIGNED flips then); the app
    container reuses 2 of its devices with no GetPreferredAllocation.  pod-resources lists only the app
    container's 2 devices, and the reconcile pass must not shrink the GROUP: the kubelet still counts
    all 4 as the pod's."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        _busy_node(c)
        c.submit("big-init", 0, split=[2], init=[4])
        kub = c.nodes["n"].kubelet
        n_pref = len(kub.preferred_calls)
        (r,) = c.schedule_pending()
        group = sorted(r.devices)
        (_, init_ids), (_, app_ids) = _calls(kub, "big-init")
        assert init_ids == tuple(group) and set(app_ids) < set(group) and len(app_ids) == 2
        assert len(kub.preferred_calls) == n_pref + 1  # only the init container asked
        assert _ann(c, "big-init").assigned and sorted(_ann(c, "big-init").group) == group
        assert c.reconcile() == 0
        assert sorted(_ann(c, "big-init").group) == group


def test_sidecar_devices_are_not_reused():
    """A sidecar (restartable init container, 1 GPU) keeps its device beside the app containers: the
    pod holds 1 + 2 devices and every container's devices are distinct."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("sc", 0, split=[2], sidecars=[1])
        pod = c.api.get_pod("default", "sc")
        assert pod_gpu_request(pod, [RES]) == 3
        assert [k for _, _, k in pod_device_steps(pod, [RES])] == ["sidecar", "app"]
        (r,) = c.schedule_pending()
        calls = _calls(c.nodes["n"].kubelet, "sc")
        assert [len(ids) for _, ids in calls] == [1, 2]
        assert sorted(i for _, ids in calls for i in ids) == sorted(r.devices)
        assert _ann(c, "sc").assigned
        assert c.reconcile() == 0  # pod-resources lists the sidecar and the app container: all 3


def test_two_multi_container_pods_assumed_together_are_admitted_in_order():
    """Two 2+2 pods bound before either is admitted: each container's request continues the pod whose
    admission is under way, so neither pod's GROUP is split across the two."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 0, split=[2, 2])
        c.submit("b", 0, split=[2, 2])
        ra, rb = c.schedule_pending(admit=False)
        kub = c.nodes["n"].kubelet
        kub.admit(c.api.get_pod("default", "a"), c.resource)
        assert _ann(c, "a").assigned and not _ann(c, "b").assigned
        kub.admit(c.api.get_pod("default", "b"), c.resource)
        for name, r in (("a", ra), ("b", rb)):
            assert sorted(int(i) for i in kub.allocated[RES][f"default/{name}"]) == sorted(r.devices)
            assert _ann(c, name).assigned and sorted(_ann(c, name).group) == sorted(r.devices)


def test_a_pod_under_admission_is_continued_before_an_older_one():
    """q (2+2) is assumed first, p (1+2) second, and the kubelet admits p first: p's 1-device
    container cannot be q's (whose next container asks 2), so p's admission is under way; p's second
    container asks 2 like q's first, and must continue p, not jump to the older q."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        groups = {"q": [0, 1, 2, 3], "p": [4, 5, 6]}
        for name, split, t in (("p", [1, 2], 200), ("q", [2, 2], 100)):  # p created first, q assumed first
            c.api.create_pod(make_pod(name, split=split, node="n",
                                      annotations=PodAssignment.assumed(groups[name], t).to_annotations()))
        kub = c.nodes["n"].kubelet
        kub.admit(c.api.get_pod("default", "p"), c.resource)
        kub.admit(c.api.get_pod("default", "q"), c.resource)
        for name, g in groups.items():
            assert sorted(int(i) for i in kub.allocated[RES][f"default/{name}"]) == g, name
            assert _ann(c, name).assigned and sorted(_ann(c, name).group) == g, name


def test_reconcile_leaves_pods_without_devices_alone():
    """A pod on the node that holds no device (no GPU request, nothing in pod-resources) is not
    stamped with an empty GROUP by the reconcile pass."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.api.create_pod(make_pod("cpu-only", node="n"))
        c.api.set_pod_phase("default", "cpu-only", "Running")
        c.submit("g", 2)
        c.schedule_pending()
        assert c.reconcile() == 0
        assert _ann(c, "cpu-only") is None


def test_single_and_multi_container_pods_of_other_sizes_do_not_steal():
    """A 4-GPU single-container pod assumed first and a 1-GPU pod assumed second, admitted in the
    other order: the 1-GPU request matches the pod whose next container asks 1, not the older GROUP."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("four", 4)
        c.submit("one", 1)
        r4, r1 = c.schedule_pending(admit=False)
        kub = c.nodes["n"].kubelet
        kub.admit(c.api.get_pod("default", "one"), c.resource)
        kub.admit(c.api.get_pod("default", "four"), c.resource)
        assert sorted(int(i) for i in kub.allocated[RES]["default/one"]) == sorted(r1.devices)
        assert sorted(int(i) for i in kub.allocated[RES]["default/four"]) == sorted(r4.devices)
        assert _ann(c, "one").assigned and _ann(c, "four").assigned


def test_kubelet_choice_outside_the_group_is_recorded_per_container():
    """A container's devices outside the GROUP (a kubelet that ignored the preferred answer): the
    GROUP is rewritten to include them, dropping GROUP devices no container got, so the extender's
    view equals the kubelet's truth without the reconcile pass."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("mm", 0, split=[2, 2])
        (r,) = c.schedule_pending(admit=False)
        group = sorted(r.devices)
        other = sorted(set(range(8)) - set(group))
        plugin = c.nodes["n"].plugin
        plugin._claim_pod(group[:2])  # the first container as preferred
        pod = plugin._claim_pod(other[:2])  # the second outside the GROUP
        assert pod is not None
        pa = _ann(c, "mm")
        assert pa.assigned and sorted(pa.group) == sorted(group[:2] + other[:2])
        assert plugin.metrics.container_claims.labels("resized")._value.get() == 1


def test_one_allocate_call_with_several_containers_still_claims_the_pod():
    """An Allocate carrying several container requests (the v1beta1 API allows it) is one step per
    container of the pod."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("old", 0, split=[2, 2])
        (r,) = c.schedule_pending(admit=False)
        g = sorted(r.devices)
        kub = c.nodes["n"].kubelet
        req = pb.AllocateRequest()
        req.container_requests.add(devices_ids=[str(i) for i in g[:2]])
        req.container_requests.add(devices_ids=[str(i) for i in g[2:]])
        resp = kub._stub(kub.plugins[c.resource], "Allocate")(req, timeout=5)
        assert len(resp.container_responses) == 2
        assert _ann(c, "old").assigned and sorted(_ann(c, "old").group) == g


def test_unannotated_multi_container_pod_is_recorded_once_complete():
    """A 2+1 pod scheduled around the extender (nodeName set, no GROUP): its containers' devices are
    collected and written as one confirmed GROUP."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        pod = c.api.create_pod(make_pod("legacy", split=[2, 1], node="n"))
        c.nodes["n"].kubelet.admit(pod, c.resource)
        pa = _ann(c, "legacy")
        got = sorted(int(i) for i in c.nodes["n"].kubelet.allocated[RES]["default/legacy"])
        assert pa.assigned and sorted(pa.group) == got and len(got) == 3


def test_time_sliced_pod_with_two_one_slice_containers():
    """A time-sliced node (2 slices per GPU): a pod of two containers with one slice each gets exactly
    its GROUP, one slice per container, and each container its own CU mask on its GPU."""
    from gpu_topology_on_k8s_amd.topology.shares import time_slice

    with SimCluster({"s": time_slice(fx.f7_mi355x(), 2)}) as c:
        c.submit("two-slices", 0, split=[1, 1], slices=True)
        (r,) = c.schedule_pending()
        kub = c.nodes["s"].kubelet
        res = c.nodes["s"].resource
        group = sorted(r.devices)
        assert len(group) == 2
        assert sorted(int(i) for i in kub.allocated[res]["default/two-slices"]) == group
        pa = _ann(c, "two-slices")
        assert pa.assigned and sorted(pa.group) == group
        calls = _calls(kub, "two-slices")
        assert [len(ids) for _, ids in calls] == [1, 1]
        masks = [dict(cr.envs).get("HSA_CU_MASK") for cr in kub.responses["default/two-slices"].container_responses]
        if len({i // 2 for i in group}) == 1:  # both slices on one GPU: the two containers' CUs are disjoint
            assert masks[0] and masks[1] and masks[0] != masks[1]


def test_swapped_init_container_pods_keep_every_held_device_annotated():
    """a = init(4) + app(2) assumed first, b = 4 GPUs assumed second, and the kubelet admits b first:
    b's call is matched to a (same count, older) and a's init call to b — the pods' annotations name
    each other's devices.  a's app container reuses 2 of the 4 devices its init container got: that
    call continues the same admission.  The annotations' union is the kubelet's, and the reconcile
    pass, which sees only a's 2 app devices in pod-resources, restores all 4 for a from the admission
    unit — no device the kubelet holds is left unannotated."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        for name, kw, g, t in (("a", dict(split=[2], init=[4]), [0, 1, 2, 3], 100), ("b", dict(split=[4]), [4, 5, 6, 7], 200)):
            c.api.create_pod(make_pod(name, node="n", annotations=PodAssignment.assumed(g, t).to_annotations(), **kw))
        kub = c.nodes["n"].kubelet
        kub.admit(c.api.get_pod("default", "b"), c.resource)
        kub.admit(c.api.get_pod("default", "a"), c.resource)
        held = {n: sorted(int(i) for i in kub.allocated[RES][f"default/{n}"]) for n in ("a", "b")}
        assert sorted(held["a"] + held["b"]) == list(range(8))
        union = sorted(_ann(c, "a").group + _ann(c, "b").group)
        assert union == list(range(8))  # the extender's view covers exactly what the kubelet holds
        c.reconcile()
        for n in ("a", "b"):
            assert sorted(_ann(c, n).group) == held[n], (n, _ann(c, n), held)


def test_swapped_init_container_pods_after_a_plugin_restart():
    """The same swap, but the plugin restarted before the reconcile pass (its admission units are
    gone): the GROUPs as written are the units — the 2 devices of b's GROUP nobody lists go to the pod
    listing the rest of it (a's app container), up to a's request of 4."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        for name, kw, g, t in (("a", dict(split=[2], init=[4]), [0, 1, 2, 3], 100), ("b", dict(split=[4]), [4, 5, 6, 7], 200)):
            c.api.create_pod(make_pod(name, node="n", annotations=PodAssignment.assumed(g, t).to_annotations(), **kw))
        kub = c.nodes["n"].kubelet
        kub.admit(c.api.get_pod("default", "b"), c.resource)
        kub.admit(c.api.get_pod("default", "a"), c.resource)
        held = {n: sorted(int(i) for i in kub.allocated[RES][f"default/{n}"]) for n in ("a", "b")}
        c.nodes["n"].plugin._unit_of.clear()  # what a restarted plugin knows
        c.reconcile()
        for n in ("a", "b"):
            assert sorted(_ann(c, n).group) == held[n], (n, _ann(c, n), held)
        assert c.reconcile() == 0


def test_a_new_pod_on_gpus_freed_before_the_status_update_is_not_the_old_one():
    """p1 ended on the kubelet (its GPUs freed) while the apiserver still shows it Running; p2, whose
    GROUP names those GPUs, is admitted next.  The kubelet asked GetPreferredAllocation with nothing to
    include, so the call reuses nothing: it is p2's, not a continuation of p1 (whose devices they were)."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.api.create_pod(make_pod("p1", gpus=2, node="n", annotations=PodAssignment.assumed([2, 3], 100).to_annotations()))
        kub = c.nodes["n"].kubelet
        kub.admit(c.api.get_pod("default", "p1"), c.resource)
        assert _ann(c, "p1").assigned
        kub.release(c.api.get_pod("default", "p1"))  # the status update lags
        c.api.create_pod(make_pod("p2", gpus=2, node="n", annotations=PodAssignment.assumed([2, 3], 200).to_annotations()))
        kub.admit(c.api.get_pod("default", "p2"), c.resource)
        assert sorted(int(i) for i in kub.allocated[RES]["default/p2"]) == [2, 3]
        assert kub.preferred_calls[-1] == ([], 2)
        assert _ann(c, "p2").assigned and sorted(_ann(c, "p2").group) == [2, 3]


def test_the_periodic_reconcile_reads_from_the_watch_cache():
    """Every node's plugin reconciles every --reconcile-interval: its pod LIST is a watch-cache read
    (resourceVersion=0), not an etcd range over all the cluster's pods; an admission still reads
    consistently.  Over HTTP the query carries resourceVersion=0."""
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer, serve_http
    from gpu_topology_on_k8s_amd.k8s.api import RestKubeAPI

    with SimCluster({"n": fx.f7_mi355x()}) as c:
        c.submit("a", 2)
        c.schedule_pending()
        before = c.api.cache_reads["Pod"]
        c.reconcile()
        assert c.api.cache_reads["Pod"] == before + 1
        c.submit("b", 2)
        c.schedule_pending()  # GetPreferredAllocation / Allocate: consistent reads
        assert c.api.cache_reads["Pod"] == before + 1
    api = FakeAPIServer()
    srv, url = serve_http(api)
    try:
        api.create_pod(make_pod("x", gpus=1, node="n"))
        got = RestKubeAPI(url).list_pods(node_name="n", cached=True)
        assert [p["metadata"]["name"] for p in got] == ["x"] and api.cache_reads["Pod"] == 1
        RestKubeAPI(url).list_pods(node_name="n")
        assert api.cache_reads["Pod"] == 1
    finally:
        srv.shutdown()
