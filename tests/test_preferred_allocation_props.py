"""GetPreferredAllocation properties (hypothesis): whatever the kubelet offers -- any available set, any
must-include subset of it, any size between the two, any mix of unhealthy devices, with or without an
annotated pod whose GROUP fits -- the answer is ``allocation_size`` distinct ids, all available, every
must-include id among them.  The kubelet rejects a pod whose preferred answer breaks any of these."""
import tempfile

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
from gpu_topology_on_k8s_amd.deviceplugin import proto as pb
from gpu_topology_on_k8s_amd.k8s import FakeAPIServer, PodAssignment
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx


@st.composite
def requests(draw):
    n = 8
    avail = sorted(draw(st.sets(st.integers(0, n - 1), min_size=1, max_size=n)))
    must = sorted(draw(st.sets(st.sampled_from(avail), max_size=len(avail))))
    size = draw(st.integers(max(1, len(must)), len(avail)))
    unhealthy = draw(st.sets(st.integers(0, n - 1), max_size=3))
    group = draw(st.none() | st.sets(st.integers(0, n - 1), min_size=1, max_size=n))
    return avail, must, size, unhealthy, group


_SOCK = tempfile.mkdtemp(prefix="gtkpa", dir="/tmp")


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(requests())
def test_preferred_answer_is_always_admissible(r):
    avail, must, size, unhealthy, group = r
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    if group is not None:  # an extender-annotated pending pod on this node
        pod = make_pod("p", gpus=len(group), node="n1")
        pod["metadata"].setdefault("annotations", {}).update(PodAssignment.assumed(sorted(group), 1_700_000_000.0).to_annotations())
        api.create_pod(pod)
    plugin = DevicePluginServer(fx.f7_mi355x(), PluginConfig(resource_name="amd.com/gpu", socket_dir=_SOCK, node_name="n1"),
                                api=api)
    for u in unhealthy:
        plugin._health[u] = False
    req = pb.PreferredAllocationRequest()
    req.container_requests.add(available_deviceIDs=[str(i) for i in avail], must_include_deviceIDs=[str(i) for i in must],
                               allocation_size=size)
    resp = plugin.GetPreferredAllocation(req, None)
    ids = [int(x) for x in resp.container_responses[0].deviceIDs]
    assert len(ids) == size and len(set(ids)) == size, (r, ids)
    assert set(ids) <= set(avail) and set(must) <= set(ids), (r, ids)
    healthy = [a for a in avail if a not in unhealthy]
    if group is None and set(must) <= set(healthy) and len(healthy) >= size:
        assert set(ids) <= set(healthy), (r, ids)  # unhealthy devices only when nothing else fits


def test_claim_rereads_when_the_pod_changed_under_it():
    """Allocate claims the oldest pending pod of the right size with a conditional patch: if the pod was
    changed in between (here the reconcile pass confirmed it with its own devices), the patch conflicts,
    the candidates are re-read, and the next pending pod is claimed instead of the confirmed one being
    overwritten."""
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    for name, group, t in (("a", [0, 1], 1_700_000_000.0), ("b", [2, 3], 1_700_000_001.0)):
        pod = make_pod(name, gpus=2, node="n1")
        pod["metadata"].setdefault("annotations", {}).update(PodAssignment.assumed(group, t).to_annotations())
        api.create_pod(pod)
    plugin = DevicePluginServer(fx.f7_mi355x(), PluginConfig(resource_name="amd.com/gpu", socket_dir=_SOCK, node_name="n1"),
                                api=api)
    real = api.patch_pod_annotations
    first = [True]

    def patch(ns, name, ann, resource_version=None):
        if first[0] and name == "a":
            first[0] = False
            real(ns, "a", {"ALIYUN_COM_GPU_ASSIGNED": "true"})  # confirmed meanwhile, on its own devices
        return real(ns, name, ann, resource_version=resource_version)

    api.patch_pod_annotations = patch
    claimed = plugin._claim_pod([4, 5])
    assert claimed["metadata"]["name"] == "b"
    a = PodAssignment.from_annotations(api.get_pod("default", "a")["metadata"]["annotations"])
    assert a.assigned and list(a.group) == [0, 1]


def test_claim_prefers_the_pod_whose_group_matches_exactly():
    """The kubelet allocated exactly what the extender annotated on the NEWER of two pending pods of the
    same size: that pod is claimed, not the older one (the oldest-same-size rule is only the fallback
    when no GROUP matches)."""
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    for name, group, t in (("old", [0, 1], 1_700_000_000.0), ("new", [2, 3], 1_700_000_005.0)):
        pod = make_pod(name, gpus=2, node="n1")
        pod["metadata"].setdefault("annotations", {}).update(PodAssignment.assumed(group, t).to_annotations())
        api.create_pod(pod)
    plugin = DevicePluginServer(fx.f7_mi355x(), PluginConfig(resource_name="amd.com/gpu", socket_dir=_SOCK, node_name="n1"),
                                api=api)
    assert plugin._claim_pod([2, 3])["metadata"]["name"] == "new"
    old = PodAssignment.from_annotations(api.get_pod("default", "old")["metadata"]["annotations"])
    assert not old.assigned and list(old.group) == [0, 1]
