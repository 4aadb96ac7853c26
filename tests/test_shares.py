"""Time-sliced GPU shares (topology/shares.py): Gaia's fractional requests (paper p.4-5 Alg. 2,
Table II; ``gaia_gpu_topology_scheduler.md:32``) on unpartitioned SPX nodes, through the model, the
annotation codec, the placement core, the device plugin and the whole cluster."""
import numpy as np
import pytest

from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
from gpu_topology_on_k8s_amd.deviceplugin import proto as pb
from gpu_topology_on_k8s_amd.k8s import Contract, PodAssignment
from gpu_topology_on_k8s_amd.k8s.annotations import decode_node_annotations, encode_node_annotations
from gpu_topology_on_k8s_amd.placement import PlacementPolicy, place_fraction, select
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.k8s.objects import make_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.identity import fractions_from_env, resolve_group
from gpu_topology_on_k8s_amd.topology.model import LinkType, Topology
from gpu_topology_on_k8s_amd.topology.shares import physical_group, share_fractions, slices_per_gpu, time_slice

C = Contract()


def _probed_f7(n=4):
    t = fx.f7_mi355x(n=n)
    bw = np.full((n, n), 70.0)
    bw[0, 1] = bw[1, 0] = 35.0  # one degraded link
    np.fill_diagonal(bw, np.nan)
    t.hbm_gbps = np.full(n, 3200.0)
    t.set_measured_bw(bw, {"method": "test", "ingress_all_gbps": [200.0] * n})
    return t


def test_time_slice_shape_links_and_costs():
    t = _probed_f7()
    v = time_slice(t, 4)
    assert v.n == 16 and slices_per_gpu(v) == 4
    assert list(v.physical) == [i // 4 for i in range(16)]
    assert all(g.vram_bytes == t.gpus[0].vram_bytes // 4 for g in v.gpus)
    assert len({g.uuid for g in v.gpus}) == 16 and all(g.bdf == t.gpus[g.physical].bdf for g in v.gpus)
    assert v.link_type[0, 1] == LinkType.INTERNAL and v.link_type[0, 4] == t.link_type[0, 1]
    # slices of one GPU exchange through its HBM: far cheaper than any link; the degraded link stays degraded
    assert v.cost[0, 1] < v.cost[0, 8] and v.cost[0, 4] == pytest.approx(t.cost[0, 1])
    assert v.cost[0, 4] > v.cost[0, 8]
    assert v.probe["ingress_all_gbps"] == [200.0] * 16 and v.probe["time_slices"] == 4
    assert time_slice(t, 1) is t


def test_time_slice_refuses_partitioned_and_double_slicing():
    with pytest.raises(ValueError, match="SPX"):
        time_slice(fx.f8_mi355x_cpx(), 2)
    with pytest.raises(ValueError, match="already"):
        time_slice(time_slice(fx.f7_mi355x(n=2), 2), 2)


def test_sliced_node_annotation_round_trip_keeps_placements():
    v = time_slice(_probed_f7(), 10)
    back = decode_node_annotations(encode_node_annotations(v, C), C)
    assert back.n == 40 and slices_per_gpu(back) == 10 and list(back.physical) == list(v.physical)
    np.testing.assert_allclose(back.cost, v.cost)
    used = list(range(20, 25))
    assert place_fraction(back, 4, used) == place_fraction(v, 4, used) == (25, 26, 27, 28)


def test_whole_gpu_request_on_a_sliced_node_takes_one_gpu():
    v = time_slice(fx.f7_mi355x(n=4), 4)
    pl = select(v, 4, used=[0], policy=PlacementPolicy(partition_aware=True))
    assert len(physical_group(v, pl.ids)) == 1 and 0 not in physical_group(v, pl.ids)


def test_share_fractions():
    v = time_slice(fx.f7_mi355x(n=2), 10)
    assert share_fractions(v, [10, 11, 12, 13]) == {1: pytest.approx(0.4)}
    assert share_fractions(v, list(range(10)) + [15]) == {0: 1.0, 1: pytest.approx(0.1)}


def test_allocate_maps_slices_to_the_physical_gpu(tmp_path):
    t = fx.f7_mi355x(n=2)
    v = time_slice(t, 10)
    plug = DevicePluginServer(v, PluginConfig(device_specs="stub", dev_root=str(tmp_path)))
    assert len(plug.devices()) == 20
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=["11", "12", "13", "14"])
    r = plug.Allocate(req, None).container_responses[0]
    envs = dict(r.envs)
    assert envs["GTK_GPU_GROUP"] == "1" and envs["GTK_GPU_BDFS"] == t.gpus[1].bdf
    assert envs["GTK_GPU_FRACTION"] == "0.4" and envs["GTK_GPU_SLICES"] == "11,12,13,14"
    assert fractions_from_env(envs) == [0.4]
    nodes = plug.device_nodes([11, 12, 13, 14])
    assert len(nodes) == len(set(nodes)) == 1 + 1 + (1 if t.gpus[1].card >= 0 else 0)
    # inside the container: the one physical GPU it sees is HIP 0
    assert resolve_group([1], bdfs=[t.gpus[1].bdf], visible_bdfs=[t.gpus[1].bdf]) == [0]


def test_table2_fragment_through_the_cluster_on_a_time_sliced_spx_node():
    """Gaia Table II on a 4-GPU SPX node advertised as 10 time slices per GPU: after 0.5 of gpu2 is
    taken, a 0.4-GPU pod and then a 0.1-GPU pod both land on gpu2 (best fit) through /filter, /sort,
    /bind, GetPreferredAllocation and Allocate, and the containers get gpu2 with their shares."""
    v = time_slice(Topology.full_mesh(n=4, numa_split=1, node_name="p4"), 10)
    with SimCluster({"p4": v}) as c:
        c.api.create_pod(make_pod("half", gpus=5, node="p4", resource=C.slice_resource,
                                  annotations=PodAssignment(list(range(20, 25)), True, 1).to_annotations()))
        c.submit("f04", 4, slices=True, annotations={C.fraction_key: "0.4"})
        r = c.schedule_pending()[0]
        assert r.error == "" and set(r.allocated) <= set(range(25, 30)) and len(r.allocated) == 4
        envs = dict(c.nodes["p4"].kubelet.responses["default/f04"].container_responses[0].envs)
        assert envs["GTK_GPU_GROUP"] == "2" and envs["GTK_GPU_FRACTION"] == "0.4"
        c.submit("f01", 1, slices=True, annotations={C.fraction_key: "0.1"})
        r = c.schedule_pending()[0]
        assert r.allocated == (29,)
        c.submit("whole", 10, slices=True)  # a whole GPU's worth of slices: all slices of one untouched GPU
        r = c.schedule_pending()[0]
        assert r.error == "" and len(physical_group(v, r.allocated)) == 1 and 2 not in physical_group(v, r.allocated)
        c.submit("gpu", 1)  # amd.com/gpu means a whole GPU: a sliced node does not offer one
        r = c.schedule_pending()[0]
        assert r.node is None and c.nodes["p4"].kubelet.rejected == []


def test_whole_gpu_and_slice_pools_stay_apart():
    """VERDICT r2 #2 (Gaia p.3 §III.A resource-pool pollution): on a cluster with one whole-GPU node
    and one time-sliced node, an unannotated ``amd.com/gpu: 1`` pod always gets a whole GPU with no
    CU mask; a ``gpu-fraction: 0.5`` pod asking for slices gets half of one GPU; every mismatch is
    named by /filter."""
    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node

    nodes = {"whole": fx.f7_mi355x(n=2), "sliced": time_slice(fx.f7_mi355x(n=2), 4)}
    with SimCluster(nodes) as c:
        assert c.nodes["sliced"].resource == C.slice_resource and c.nodes["whole"].resource == C.resource_name
        alloc = {n: c.api.get_node(n)["status"]["allocatable"] for n in nodes}
        assert alloc["whole"] == {C.resource_name: "2"} and alloc["sliced"] == {C.slice_resource: "8"}
        for i in range(2):  # the whole-GPU node's two GPUs, each with no CU mask
            c.submit(f"g{i}", 1)
            r = c.schedule_pending()[0]
            assert r.node == "whole", r
            envs = dict(c.nodes["whole"].kubelet.responses[f"default/g{i}"].container_responses[0].envs)
            assert "HSA_CU_MASK" not in envs and "GTK_GPU_FRACTION" not in envs
        c.submit("g2", 1)  # no whole GPU left anywhere: pending, never a quarter GPU on the sliced node
        r = c.schedule_pending()[0]
        assert r.node is None
        c.api.delete_pod("default", "g2")
        c.submit("half", 2, slices=True, annotations={C.fraction_key: "0.5"})
        r = c.schedule_pending()[0]
        assert r.node == "sliced" and len(physical_group(nodes["sliced"], r.allocated)) == 1
        envs = dict(c.nodes["sliced"].kubelet.responses["default/half"].container_responses[0].envs)
        assert envs["GTK_GPU_FRACTION"] == "0.5" and envs["HSA_CU_MASK"].startswith("0:")

    api = FakeAPIServer()
    for n, t in nodes.items():
        api.create_node(make_node(n, annotations=encode_node_annotations(t, C)))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    gpu = api.create_pod(make_pod("gpu", gpus=1))
    ok, failed = ext.filter(gpu, ["whole", "sliced"])
    assert ok == ["whole"] and "amd.com/gpu-slice" in failed["sliced"] and "whole GPUs" in failed["sliced"]
    sl = api.create_pod(make_pod("sl", gpus=1, resource=C.slice_resource))
    ok, failed = ext.filter(sl, ["whole", "sliced"])
    assert ok == ["sliced"] and "no time slices" in failed["whole"]
    frac = api.create_pod(make_pod("frac", gpus=1, annotations={C.fraction_key: "0.25"}))  # fraction, wrong pool
    ok, failed = ext.filter(frac, ["whole", "sliced"])
    assert ok == [] and "partitioned" in failed["whole"] and "amd.com/gpu-slice" in failed["sliced"]
    both = make_pod("both", gpus=1)
    both["spec"]["containers"].append({"name": "c1", "resources": {"limits": {C.slice_resource: "1"}}})
    both = api.create_pod(both)
    ok, failed = ext.filter(both, ["whole", "sliced"])
    assert ok == [] and "both" in failed["whole"]


def test_gpu_reset_holds_every_slice_of_the_gpu():
    v = time_slice(fx.f7_mi355x(n=2), 4)
    plug = DevicePluginServer(v, PluginConfig())
    plug.gpu_event(5, "GPU_PRE_RESET", "test")
    assert [d.health for d in plug.devices()] == [pb.HEALTHY] * 4 + [pb.UNHEALTHY] * 4
    plug.gpu_event(5, "GPU_POST_RESET", "test")
    assert all(d.health == pb.HEALTHY for d in plug.devices())


def test_slice_compute_units_and_cu_mask():
    from gpu_topology_on_k8s_amd.topology.shares import cu_mask_env, slice_cus

    v = time_slice(fx.f7_mi355x(n=2), 4)  # fixtures carry no CU count: MI355X's 256
    assert slice_cus(v, 0) == list(range(0, 64)) and slice_cus(v, 7) == list(range(192, 256))
    assert cu_mask_env(v, [5, 6]) == "0:64-191"  # the pod sees GPU 1 as its only device
    assert cu_mask_env(v, [0, 2]) == "0:0-63,128-191"
    assert cu_mask_env(v, [0, 1, 2, 3, 7]) == "1:192-255"  # GPU 0 whole (no mask), a quarter of GPU 1
    assert cu_mask_env(fx.f7_mi355x(n=2), [0]) == ""
    v8 = time_slice(Topology.full_mesh(n=1), 8)
    v8.gpus[0].cus = 240  # e.g. a part with harvested CUs: runs of 30
    assert slice_cus(v8, 0) == list(range(0, 30))


def test_allocate_sets_cu_mask_after_pod_env(tmp_path):
    from gpu_topology_on_k8s_amd.k8s.objects import make_pod as mk

    v = time_slice(fx.f7_mi355x(n=2), 4)
    plug = DevicePluginServer(v, PluginConfig(device_specs="stub", dev_root=str(tmp_path)))
    pod = mk("p", gpus=2, annotations={f"{C.prefix}/rccl-env": "HSA_CU_MASK=0:0-255;NCCL_MIN_NCHANNELS=8"})
    r = plug._container_response([4, 5], plug._rccl_env(pod))
    assert r.envs["HSA_CU_MASK"] == "0:0-127" and r.envs["NCCL_MIN_NCHANNELS"] == "8"
    off = DevicePluginServer(v, PluginConfig(device_specs="stub", dev_root=str(tmp_path), share_cu_mask=False))
    assert "HSA_CU_MASK" not in off._container_response([4, 5], {}).envs


def test_cdi_mode_names_each_physical_gpu_once(tmp_path):
    v = time_slice(fx.f7_mi355x(n=2), 4)
    plug = DevicePluginServer(v, PluginConfig(device_specs="cdi", cdi_dir=str(tmp_path)))
    r = plug._container_response([4, 5, 6], {})
    assert [d.name for d in r.cdi_devices] == ["amd.com/gpu=4"] and r.envs["GTK_GPU_GROUP"] == "1"
    r = plug._container_response([2, 3, 4], {})
    assert [d.name for d in r.cdi_devices] == ["amd.com/gpu=0", "amd.com/gpu=4"]
    assert r.envs["GTK_GPU_FRACTION"] == "0.5,0.25" and r.envs["HSA_CU_MASK"] == "0:128-255;1:0-63"


def test_time_slice_keeps_explicit_pair_costs():
    """A topology priced explicitly (the paper's PCIe tree, F4 costs) keeps those costs between GPUs;
    slices of one GPU are the cheapest pairs."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench"))
    import cluster_trace as ct

    t = ct._tree_node(0)
    v = time_slice(t, 2)
    for a in range(8):
        for b in range(8):
            if a != b:
                assert v.cost[2 * a, 2 * b + 1] == pytest.approx(t.cost[a, b])
    assert v.cost[0, 1] < v.cost[0, 2]


def test_gpu_memory_sizes_the_share():
    """``gpu-memory`` sizes a share by HBM: on a 4-slice MI355X node (72 GB per slice) 100 GB needs
    2 slices of one GPU; the pod must ask for that count; on whole-GPU nodes it only has to fit."""
    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node

    api = FakeAPIServer()
    api.create_node(make_node("s", annotations=encode_node_annotations(time_slice(fx.f7_mi355x(), 4), C),
                              capacity={C.slice_resource: "32"}))
    api.create_node(make_node("w", annotations=encode_node_annotations(fx.f7_mi355x(), C), capacity={C.resource_name: "8"}))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    two = api.create_pod(make_pod("m2", gpus=2, resource=C.slice_resource, annotations={C.memory_key: "100G"}))
    ok, failed = ext.filter(two, ["s", "w"])
    assert ok == ["s"] and "no time slices" in failed["w"]
    d = ext.bind("default", "m2", two["metadata"]["uid"], "s")
    assert len(physical_group(ext.cache.get("s").topology, d.ids)) == 1 and d.policy == "fragment"
    whole2 = api.create_pod(make_pod("w2", gpus=2, annotations={C.memory_key: "100G"}))
    ok, failed = ext.filter(whole2, ["s", "w"])
    assert ok == ["w"]  # whole GPUs: simply two of them (each holds 100 GB)
    bad = api.create_pod(make_pod("m1", gpus=1, resource=C.slice_resource, annotations={C.memory_key: "100G"}))
    ok, failed = ext.filter(bad, ["s", "w"])
    assert ok == [] and "2 of 4" in failed["s"]
    big = api.create_pod(make_pod("huge", gpus=1, annotations={C.memory_key: "400Gi"}))
    ok, failed = ext.filter(big, ["w"])
    assert ok == [] and "exceeds" in failed["w"]
    big_s = api.create_pod(make_pod("huge-s", gpus=4, resource=C.slice_resource, annotations={C.memory_key: "400Gi"}))
    ok, failed = ext.filter(big_s, ["s"])
    assert ok == [] and "exceeds" in failed["s"]


def test_share_gauge_per_gpu():
    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node

    api = FakeAPIServer()
    api.create_node(make_node("s", annotations=encode_node_annotations(time_slice(fx.f7_mi355x(n=2), 4), C),
                              capacity={C.slice_resource: "8"}))
    api.create_pod(make_pod("q", gpus=3, node="s", resource=C.slice_resource,
                            annotations=PodAssignment([4, 5, 6], True, 1).to_annotations()))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    ext.cache.sync_all()
    text = ext.metrics.exposition().decode()
    assert 'gtk_extender_gpu_share_used{gpu="1",node="s"} 0.75' in text
    assert 'gtk_extender_gpu_share_used{gpu="0",node="s"} 0.0' in text


def test_reset_of_a_sliced_gpu_is_one_event_and_one_publish():
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node

    api = FakeAPIServer()
    api.create_node(make_node("n"))
    plug = DevicePluginServer(time_slice(fx.f7_mi355x(n=2), 4), PluginConfig(node_name="n"), api=api)
    calls = []
    orig = api.patch_node
    api.patch_node = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    plug.gpu_event(6, "GPU_PRE_RESET", "test")
    resets = [e for e in api.events if e["reason"] == "GPUUnhealthy"]
    assert len(resets) == 1 and "4,5,6,7" in resets[0]["message"] and len(calls) == 1


def test_node_label_devices_per_gpu():
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node

    api = FakeAPIServer()
    for name, topo in (("s", time_slice(fx.f7_mi355x(n=2), 4)), ("w", fx.f7_mi355x(n=2)), ("c", fx.f8_mi355x_cpx())):
        api.create_node(make_node(name))
        DevicePluginServer(topo, PluginConfig(node_name=name), api=api)._publish_node()
    labels = {n: api.get_node(n)["metadata"]["labels"][C.label_slices] for n in ("s", "w", "c")}
    assert labels == {"s": "4", "w": "1", "c": "8"}


def test_gpu_memory_on_a_node_without_device_sizes_is_refused_with_the_reason():
    """A sliced node whose topology carries no device memory sizes cannot size a ``gpu-memory`` request:
    /filter names why for that node instead of failing the verb."""
    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node

    t = time_slice(fx.f7_mi355x(), 4)
    for g in t.gpus:
        g.vram_bytes = 0
    api = FakeAPIServer()
    api.create_node(make_node("s", annotations=encode_node_annotations(t, C), capacity={C.slice_resource: "32"}))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    pod = api.create_pod(make_pod("m2", gpus=2, resource=C.slice_resource, annotations={C.memory_key: "100G"}))
    ok, failed = ext.filter(pod, ["s"])
    assert ok == [] and "cannot be sized" in failed["s"], failed


def test_small_pods_pack_onto_the_fuller_node():
    """Node-level best fit: with the same placement quality on both nodes, a 2-GPU pod goes to the node
    that already runs work, keeping the empty node whole for an 8-GPU job."""
    from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node

    api = FakeAPIServer()
    for n in ("empty", "busy"):
        api.create_node(make_node(n, annotations=encode_node_annotations(fx.f7_mi355x(), C), capacity={C.resource_name: "8"}))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    first = api.create_pod(make_pod("first", gpus=4))
    ext.bind("default", "first", first["metadata"]["uid"], "busy")
    pod = api.create_pod(make_pod("small", gpus=2))
    scores = dict(ext.prioritize(pod, ["empty", "busy"]))
    assert scores["busy"] > scores["empty"], scores
