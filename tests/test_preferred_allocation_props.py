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
