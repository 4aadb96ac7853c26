"""Device health from RAS signals (deviceplugin/health.py): the policy, the
monitor's transitions, and the plugin re-advertising a device that turns Unhealthy."""
import dataclasses

from gpu_topology_on_k8s_amd.deviceplugin.health import HealthMonitor, HealthPolicy, device_problems
from gpu_topology_on_k8s_amd.topology.discovery import fake_topology
from gpu_topology_on_k8s_amd.topology.model import GPUInfo


def _gpu(**kw):
    base = dict(index=0, ecc_uncorrectable=3, ecc_correctable=10, bad_pages=2, bad_page_threshold=64, xgmi_links_up=7)
    base.update(kw)
    return GPUInfo(**base)


def test_policy_signals():
    base = _gpu()
    assert device_problems(_gpu(), base) == []
    assert device_problems(_gpu(ecc_correctable=500), base) == []  # correctable errors alone are not fatal
    assert "uncorrectable" in device_problems(_gpu(ecc_uncorrectable=4), base)[0]
    assert "retired pages" in device_problems(_gpu(bad_pages=64), base)[0]
    assert "xGMI" in device_problems(_gpu(xgmi_links_up=6), base)[0]
    assert device_problems(_gpu(healthy=False), base)
    # unreadable signals (-1) never count as failures
    assert device_problems(_gpu(ecc_uncorrectable=-1, bad_pages=-1, xgmi_links_up=-1), base) == []
    assert device_problems(_gpu(ecc_uncorrectable=9), _gpu(ecc_uncorrectable=-1)) == []
    assert device_problems(_gpu(xgmi_links_up=6), base, HealthPolicy(xgmi_links=False)) == []


def test_monitor_transitions_and_vanished_device():
    topo = fake_topology(4)
    for g in topo.gpus:
        g.ecc_uncorrectable, g.xgmi_links_up = 0, 3
    state = {"topo": topo}

    def rediscover():
        return state["topo"]

    mon = HealthMonitor(topo, rediscover)
    assert mon(topo) == {0: True, 1: True, 2: True, 3: True}
    bad = fake_topology(4)
    for g in bad.gpus:
        g.ecc_uncorrectable, g.xgmi_links_up = 0, 3
    bad.gpus[2] = dataclasses.replace(bad.gpus[2], ecc_uncorrectable=1)
    bad.gpus[3] = dataclasses.replace(bad.gpus[3], xgmi_links_up=2)
    state["topo"] = bad
    assert mon(topo) == {0: True, 1: True, 2: False, 3: False}
    assert "uncorrectable" in mon.reasons[2][0] and "xGMI" in mon.reasons[3][0]
    state["topo"] = topo  # links retrain, counters as at start
    assert all(mon(topo).values()) and mon.reasons[3] == []
    shrunk = fake_topology(3)
    for g in shrunk.gpus:
        g.ecc_uncorrectable, g.xgmi_links_up = 0, 3
    state["topo"] = shrunk
    res = mon(topo)
    assert res[3] is False and "vanished" in mon.reasons[3][0]


def test_json_roundtrip_keeps_ras_fields():
    from gpu_topology_on_k8s_amd.topology.model import Topology

    t = fake_topology(2)
    t.gpus[1].ecc_uncorrectable = 5
    t.gpus[1].bad_page_threshold = 64
    u = Topology.from_json(t.to_json())
    assert u.gpus[1].ecc_uncorrectable == 5 and u.gpus[1].bad_page_threshold == 64


def test_link_loss_degrade_republishes_pair_class():
    """--xgmi-link-loss degrade: the GPU stays Healthy, the re-discovered pair class is republished and
    its stale measurement dropped, so the extender prices the pair as PCIe and avoids it."""
    import numpy as np

    from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
    from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.annotations import decode_node_annotations
    from gpu_topology_on_k8s_amd.k8s.objects import make_node
    from gpu_topology_on_k8s_amd.placement import select
    from gpu_topology_on_k8s_amd.topology import fixtures as fx
    from gpu_topology_on_k8s_amd.topology.model import LinkType

    topo = fx.f7_mi355x(link_gbps=70.0)
    fresh = fx.f7_mi355x(link_gbps=70.0)
    fresh.link_type[0, 5] = fresh.link_type[5, 0] = int(LinkType.PCIE_SYS)
    fresh.hops[0, 5] = fresh.hops[5, 0] = 3
    fresh.gpus[0].xgmi_links_up = fresh.gpus[5].xgmi_links_up = 6
    mon = HealthMonitor(topo, lambda: fresh, HealthPolicy(xgmi_links=False))
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    plug = DevicePluginServer(topo, PluginConfig(node_name="n1"), api=api, health_fn=mon)
    assert all(mon(topo).values())  # nobody goes Unhealthy
    new = mon.relink(plug.topology)
    assert new is not None and new.probe["relinked"] == [(0, 5)] and np.isnan(new.bw_gbps[0, 5])
    plug.update_topology(new)
    pub = decode_node_annotations(api.get_node("n1")["metadata"]["annotations"], Contract())
    assert LinkType(int(pub.link_type[0, 5])) == LinkType.PCIE_SYS and pub.cost[0, 5] > 4 * pub.cost[0, 1]
    assert set(select(pub, 2, used=[1, 2, 3, 4, 6, 7]).ids) == {0, 5}  # only pair left: still schedulable
    assert mon.relink(new) is None  # nothing changed since


def test_partition_switch_requests_restart():
    """a compute-partition switch (SPX -> CPX) changes the device set; the plugin flags a
    restart (the daemon exits 75 so the DaemonSet restarts it) instead of advertising stale IDs."""
    import time

    from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
    from gpu_topology_on_k8s_amd.k8s.objects import make_node
    from gpu_topology_on_k8s_amd.topology import fixtures as fx

    state = {"topo": fx.f7_mi355x()}
    mon = HealthMonitor(fx.f7_mi355x(), lambda: state["topo"])
    assert mon(fx.f7_mi355x()) and mon.layout_changed() is None
    state["topo"] = fx.f8_mi355x_cpx()
    mon(fx.f7_mi355x())
    assert "device count 8 -> 64" in mon.layout_changed()
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    import tempfile

    d = tempfile.mkdtemp(prefix="gtkh", dir="/tmp")
    plug = DevicePluginServer(fx.f7_mi355x(), PluginConfig(node_name="n1", socket_dir=d, health_interval=0.05), api=api,
                              health_fn=HealthMonitor(fx.f7_mi355x(), lambda: state["topo"]))
    plug.start(register=False)
    try:
        assert plug.layout_change.wait(5) and "64" in plug.layout_change_reason
        assert any(e["reason"] == "GPULayoutChanged" for e in api.events)
    finally:
        plug.stop()
