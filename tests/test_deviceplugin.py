"""Device plugin against the fake kubelet over real gRPC unix sockets (SURVEY.md §4 "Unit: device plugin")."""
import shutil
import tempfile
import time

import grpc
import pytest

import os

from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, FakeKubelet, PluginConfig, placeholder_dev_tree
from gpu_topology_on_k8s_amd.deviceplugin import proto as pb
from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.k8s import ANN_ASSIGNED, ANN_ASSUME_TIME, ANN_GROUP, Contract, FakeAPIServer, PodAssignment
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx

RES = "amd.com/gpu"


@pytest.fixture
def sockdir():
    d = tempfile.mkdtemp(prefix="gtkdp", dir="/tmp")  # unix socket paths must stay < 108 bytes
    yield d
    shutil.rmtree(d, ignore_errors=True)


@pytest.fixture
def node(sockdir):
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    kubelet = FakeKubelet(sockdir, node_name="n1", api=api)
    kubelet.start()
    topo = fx.f7_mi355x()
    dev = placeholder_dev_tree(os.path.join(sockdir, "dev"), topo)
    plugin = DevicePluginServer(topo, PluginConfig(resource_name=RES, socket_dir=sockdir, node_name="n1", dev_root=dev), api=api)
    plugin.start()
    kubelet.wait_for(RES)
    yield api, kubelet, plugin, topo
    plugin.stop()
    kubelet.stop()


def _wait(pred, timeout=5.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_register_and_list_and_watch(node):
    api, kubelet, plugin, topo = node
    p = kubelet.plugins[RES]
    assert sorted(p.devices, key=int) == [str(i) for i in range(8)]
    assert set(p.devices.values()) == {pb.HEALTHY}
    opts = kubelet.options(RES)
    assert opts.get_preferred_allocation_available and not opts.pre_start_required
    n = api.get_node("n1")
    assert n["status"]["capacity"][RES] == "8"  # kubelet published capacity (diagram step 2)
    c = Contract(resource_name=RES)
    assert n["metadata"]["annotations"]["GPU_XGMI_0_1"] == "xGMI 1 hop"  # design.md:76-82 shape
    assert c.topology_key in n["metadata"]["annotations"]
    assert n["metadata"]["labels"][c.label_model] == "MI355X"


def test_device_numa_topology_reported(node):
    _, _, plugin, _ = node
    devs = plugin.devices()
    assert [d.topology.nodes[0].ID for d in devs] == [0, 0, 0, 0, 1, 1, 1, 1]


def test_health_change_is_streamed(node):
    api, kubelet, plugin, _ = node
    plugin.set_health(5, False)
    assert _wait(lambda: kubelet.plugins[RES].devices.get("5") == pb.UNHEALTHY)
    assert _wait(lambda: api.get_node("n1")["status"]["allocatable"][RES] == "7")
    assert "5" not in kubelet.available(RES)
    plugin.set_health(5, True)
    assert _wait(lambda: kubelet.plugins[RES].devices.get("5") == pb.HEALTHY)


def test_allocate_follows_extender_group_and_flips_assigned(node):
    """design.md:236-246: Allocate reads GROUP, injects devices, sets ASSIGNED=true + fresh ASSUME_TIME."""
    api, kubelet, plugin, topo = node
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    pod = api.create_pod(make_pod("train", gpus=4))
    d = ext.bind("default", "train", pod["metadata"]["uid"], "n1")
    pod = api.get_pod("default", "train")
    resp = kubelet.admit(pod, RES)
    assert kubelet.allocated[RES]["default/train"] == tuple(str(i) for i in d.ids)  # preferred == GROUP
    c = resp.container_responses[0]
    paths = [x.container_path for x in c.devices]
    assert paths[0] == "/dev/kfd"
    for i in d.ids:
        assert f"/dev/dri/renderD{128 + i}" in paths and f"/dev/dri/card{i}" in paths
    assert all(x.permissions == "rw" for x in c.devices)
    assert all(x.host_path.startswith(plugin.cfg.dev_root) and os.path.exists(x.host_path) for x in c.devices)
    assert c.envs["GTK_GPU_GROUP"] == ",".join(map(str, d.ids))
    assert c.envs["GTK_GPU_BDFS"] == ",".join(topo.gpus[i].bdf for i in d.ids)  # GROUP -> HIP ordinal inside the pod
    assert "NVIDIA_VISIBLE_DEVICES" not in c.envs
    ann = api.get_pod("default", "train")["metadata"]["annotations"]
    assert ann[ANN_ASSIGNED] == "true" and ann[ANN_GROUP] == ",".join(map(str, d.ids))
    assert int(ann[ANN_ASSUME_TIME]) > 0


def test_preferred_allocation_without_pod_uses_placement_core(node):
    _, kubelet, plugin, _ = node
    req = pb.PreferredAllocationRequest()
    req.container_requests.add(available_deviceIDs=[str(i) for i in range(8)], allocation_size=4)
    req.container_requests.add(available_deviceIDs=["1", "2", "5", "6"], must_include_deviceIDs=["5"], allocation_size=2)
    resp = kubelet._stub(kubelet.plugins[RES], "GetPreferredAllocation")(req, timeout=5)
    assert list(resp.container_responses[0].deviceIDs) in (["0", "1", "2", "3"], ["4", "5", "6", "7"])
    assert list(resp.container_responses[1].deviceIDs) == ["5", "6"]


def test_allocate_for_pod_scheduled_around_extender(node):
    api, kubelet, plugin, _ = node
    pod = api.create_pod(make_pod("legacy", gpus=2, node="n1"))
    kubelet.admit(pod, RES)
    ann = api.get_pod("default", "legacy")["metadata"]["annotations"]
    pa = PodAssignment.from_annotations(ann)
    assert pa.assigned and len(pa.group) == 2  # recorded so the extender sees the usage


def test_allocate_rejects_unknown_and_unhealthy(node):
    _, kubelet, plugin, _ = node
    stub = kubelet._stub(kubelet.plugins[RES], "Allocate")
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=["42"])
    with pytest.raises(grpc.RpcError) as ei:
        stub(req, timeout=5)
    assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    plugin.set_health(0, False)
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=["0"])
    with pytest.raises(grpc.RpcError) as ei:
        stub(req, timeout=5)
    assert ei.value.code() == grpc.StatusCode.FAILED_PRECONDITION


def test_multi_container_pod(node):
    api, kubelet, plugin, _ = node
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
    pod = make_pod("mc", gpus=0, containers=2)
    for c in pod["spec"]["containers"]:
        c["resources"] = {"limits": {RES: "2"}}
    pod = api.create_pod(pod)
    d = ext.bind("default", "mc", pod["metadata"]["uid"], "n1")
    assert len(d.ids) == 4
    resp = kubelet.admit(api.get_pod("default", "mc"), RES)  # one GetPreferredAllocation + Allocate per container
    assert len(resp.container_responses) == 2
    assert [len(ids) for _, _, ids in kubelet.allocate_calls] == [2, 2]
    pa = PodAssignment.from_annotations(api.get_pod("default", "mc")["metadata"]["annotations"])
    assert pa.assigned and sorted(pa.group) == sorted(d.ids)
    assert sorted(int(i) for i in kubelet.allocated[RES]["default/mc"]) == sorted(d.ids)


def test_rccl_env_passthrough(node):
    api, kubelet, plugin, _ = node
    c = Contract(resource_name=RES)
    pod = api.create_pod(make_pod("env", gpus=1, node="n1", annotations={
        f"{c.prefix}/rccl-env": "NCCL_MIN_NCHANNELS=32\nLD_PRELOAD=/evil.so\nRCCL_MSCCL_ENABLE=0",
        **PodAssignment.assumed([3], 1).to_annotations()}))
    resp = kubelet.admit(pod, RES)
    envs = resp.container_responses[0].envs
    assert envs["NCCL_MIN_NCHANNELS"] == "32" and envs["RCCL_MSCCL_ENABLE"] == "0"
    assert "LD_PRELOAD" not in envs  # only RCCL/HIP tuning variables pass


def test_containers_get_the_ipc_mode_rccl_needs(node, monkeypatch):
    """Every allocated container gets HSA_ENABLE_IPC_MODE_LEGACY as the plugin has it (0 in the rendered
    manifests: dma-buf IPC handles, which multi-process RCCL needs on these hosts); a pod's rccl-env may
    override it, and an empty setting hands none."""
    api, kubelet, plugin, _ = node
    c = Contract(resource_name=RES)
    plugin.cfg.container_ipc_mode = "0"
    pod = api.create_pod(make_pod("ipc", gpus=2, node="n1", annotations=PodAssignment.assumed([0, 1], 1).to_annotations()))
    assert kubelet.admit(pod, RES).container_responses[0].envs["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    pod = api.create_pod(make_pod("own", gpus=1, node="n1", annotations={
        f"{c.prefix}/rccl-env": "HSA_ENABLE_IPC_MODE_LEGACY=1", **PodAssignment.assumed([2], 1).to_annotations()}))
    assert kubelet.admit(pod, RES).container_responses[0].envs["HSA_ENABLE_IPC_MODE_LEGACY"] == "1"
    plugin.cfg.container_ipc_mode = ""
    pod = api.create_pod(make_pod("none", gpus=1, node="n1", annotations=PodAssignment.assumed([3], 1).to_annotations()))
    assert "HSA_ENABLE_IPC_MODE_LEGACY" not in kubelet.admit(pod, RES).container_responses[0].envs
    from gpu_topology_on_k8s_amd.deviceplugin.plugin import PluginConfig as PC

    monkeypatch.setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    assert PC().container_ipc_mode == "0" and PC(container_ipc_mode="").container_ipc_mode == ""
    monkeypatch.delenv("HSA_ENABLE_IPC_MODE_LEGACY")
    assert PC().container_ipc_mode == ""


def test_kubelet_restart_triggers_reregistration(node):
    api, kubelet, plugin, _ = node
    assert plugin.registered == 1
    kubelet.restart()
    assert _wait(lambda: plugin.registered >= 2, timeout=10)
    kubelet.wait_for(RES)
    assert len(kubelet.plugins[RES].devices) == 8


def test_health_fn_polling(sockdir):
    api = FakeAPIServer()
    api.create_node(make_node("n2"))
    kubelet = FakeKubelet(sockdir, node_name="n2", api=api)
    kubelet.start()
    state = {2: True}
    plugin = DevicePluginServer(fx.f7_mi355x(n=4), PluginConfig(resource_name=RES, socket_dir=sockdir, node_name="n2",
                                                                 health_interval=0.05),
                                api=api, health_fn=lambda t: dict(state))
    plugin.start()
    try:
        kubelet.wait_for(RES)
        state[2] = False  # e.g. amdsmi reports an xGMI/RAS fault
        assert _wait(lambda: kubelet.plugins[RES].devices.get("2") == pb.UNHEALTHY)
    finally:
        plugin.stop()
        kubelet.stop()


def _measured(n=4, bw=60.0, degrade=None):
    import numpy as np

    t = fx.f7_mi355x(n=n)
    m = np.full((t.n, t.n), bw)
    np.fill_diagonal(m, np.nan)
    if degrade:
        i, j, f = degrade
        m[i, j] = m[j, i] = bw * f
    t.set_measured_bw(m, {"method": "p2p_read_lds", "preset": "quick"})
    return t


def test_reprobe_republishes_only_when_idle_and_changed():
    """Idle-time link re-probe: a degraded pair measured while no pod holds a device
    is republished on the node; a re-probe within tolerance or a busy node changes nothing."""
    import json

    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    base = _measured()
    results = [_measured(bw=61.0), _measured(degrade=(0, 3, 0.5))]
    plug = DevicePluginServer(base, PluginConfig(node_name="n1", reprobe_tolerance=0.15), api=api,
                              reprobe_fn=lambda: results.pop(0))
    plug._publish_node()
    assert plug.node_idle()
    assert plug.reprobe() is False  # +1.7 %: within tolerance
    assert plug.reprobe() is True  # pair (0,3) at half speed
    from gpu_topology_on_k8s_amd.topology.model import Topology

    topo = Topology.from_json(api.get_node("n1")["metadata"]["annotations"][Contract().topology_key])
    assert topo.bw_gbps[0][3] == 30.0 and plug.republished == 1 and plug.reprobes == 2
    # a pod holding devices makes the node busy: the monitor must not probe
    api.create_pod(make_pod("busy", gpus=2, node="n1", annotations=PodAssignment.assumed((0, 1), 1).to_annotations()))
    assert not plug.node_idle()
    assert DevicePluginServer.link_change(base, _measured()) == 0.0


def test_reprobe_runs_from_the_monitor_loop():
    api = FakeAPIServer()
    api.create_node(make_node("n2"))
    calls = []

    def fn():
        calls.append(1)
        return _measured(degrade=(1, 2, 0.3))

    sockdir = tempfile.mkdtemp(prefix="gtkp", dir="/tmp")
    plug = DevicePluginServer(_measured(), PluginConfig(node_name="n2", socket_dir=sockdir, reprobe_interval=0.3), api=api,
                              reprobe_fn=fn)
    try:
        plug.start(register=False)
        t0 = time.time()
        while plug.republished == 0 and time.time() - t0 < 10:
            time.sleep(0.1)
        assert calls and plug.republished >= 1
    finally:
        plug.stop()
        shutil.rmtree(sockdir, ignore_errors=True)


def test_cdi_mode_allocates_by_cdi_name_and_writes_the_spec(sockdir):
    """--device-specs cdi: Allocate returns `amd.com/gpu=<GROUP index>` names, no DeviceSpecs; the spec
    the plugin wrote resolves every name to existing render/card nodes plus the common /dev/kfd."""
    import json

    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    cdi = os.path.join(sockdir, "cdi")
    kubelet = FakeKubelet(sockdir, node_name="n1", api=api, cdi_dir=cdi)
    kubelet.start()
    topo = fx.f7_mi355x()
    dev = placeholder_dev_tree(os.path.join(sockdir, "dev"), topo)
    plugin = DevicePluginServer(topo, PluginConfig(resource_name=RES, socket_dir=sockdir, node_name="n1", dev_root=dev,
                                                   device_specs="cdi", cdi_dir=cdi), api=api)
    plugin.start()
    try:
        kubelet.wait_for(RES)
        spec = json.load(open(os.path.join(cdi, "amd.com-gpu.json")))
        assert spec["kind"] == "amd.com/gpu" and len(spec["devices"]) == 8
        assert spec["containerEdits"]["deviceNodes"][0]["path"] == "/dev/kfd"
        ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
        pod = api.create_pod(make_pod("cdi", gpus=2))
        d = ext.bind("default", "cdi", pod["metadata"]["uid"], "n1")
        resp = kubelet.admit(api.get_pod("default", "cdi"), RES)
        c = resp.container_responses[0]
        assert [x.name for x in c.cdi_devices] == [f"amd.com/gpu={i}" for i in d.ids] and len(c.devices) == 0
        assert c.envs["GTK_GPU_GROUP"] == ",".join(map(str, d.ids))
        # a runtime with the spec gone cannot create the container
        os.unlink(os.path.join(cdi, "amd.com-gpu.json"))
        from gpu_topology_on_k8s_amd.deviceplugin.kubelet import AdmissionError

        with pytest.raises(AdmissionError, match="unresolvable CDI"):
            kubelet.admit(api.create_pod(make_pod("cdi2", gpus=1)), RES)
        plugin.update_topology(topo)  # republish rewrites the spec
        assert os.path.exists(os.path.join(cdi, "amd.com-gpu.json"))
    finally:
        plugin.stop()
        kubelet.stop()
    with pytest.raises(ValueError):
        PluginConfig(device_specs="nvidia")


def test_allocate_sets_nccl_ib_hca_to_the_gpus_own_nics(sockdir, tmp_path):
    """Multi-node RCCL: Allocate points NCCL_IB_HCA at the NIC behind each allocated GPU's PCIe switch."""
    from gpu_topology_on_k8s_amd._native import available, load
    from gpu_topology_on_k8s_amd.topology.discovery import from_native

    if not available("_topo"):
        pytest.skip("_topo not built")
    p = fx.write_fake_kfd_sysfs(str(tmp_path), nics=True)
    topo = from_native(load("_topo").discover_sysfs(p["kfd"], p["drm"], p["pci"], p["node"], p["ib"]))
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    kubelet = FakeKubelet(sockdir, node_name="n1", api=api)
    kubelet.start()
    dev = placeholder_dev_tree(os.path.join(sockdir, "dev"), topo)
    plugin = DevicePluginServer(topo, PluginConfig(resource_name=RES, socket_dir=sockdir, node_name="n1", dev_root=dev), api=api)
    plugin.start()
    try:
        kubelet.wait_for(RES)
        ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0))
        pod = api.create_pod(make_pod("mn", gpus=2))
        d = ext.bind("default", "mn", pod["metadata"]["uid"], "n1")
        c = kubelet.admit(api.get_pod("default", "mn"), RES).container_responses[0]
        want = [f"ionic_{topo.gpus[i].physical}" for i in d.ids]
        assert c.envs["GTK_NICS"] == ",".join(want) and c.envs["NCCL_IB_HCA"] == "=" + ",".join(want)
    finally:
        plugin.stop()
        kubelet.stop()


def test_liveness_reports_a_wedged_monitor_and_failing_registration(sockdir):
    """/healthz is the DaemonSet's livenessProbe: 200 while the plugin serves; 503 with the reason when
    the monitor loop is stuck (here in a health poll that never returns, as a hung driver call would
    be) or re-registration after a kubelet restart keeps failing, so the kubelet restarts the plugin."""
    import threading

    import requests

    from gpu_topology_on_k8s_amd.deviceplugin import serve_metrics

    api = FakeAPIServer()
    api.create_node(make_node("n3"))
    kubelet = FakeKubelet(sockdir, node_name="n3", api=api)
    kubelet.start()
    release = threading.Event()
    wedge = threading.Event()

    def health(t):
        if wedge.is_set():
            release.wait(30)  # a driver call that does not come back
        return {g.index: True for g in t.gpus}

    plugin = DevicePluginServer(fx.f7_mi355x(n=4), PluginConfig(resource_name=RES, socket_dir=sockdir, node_name="n3",
                                                                 health_interval=0.05), api=api, health_fn=health)
    plugin.metrics.liveness = plugin.liveness
    srv, base = serve_metrics(plugin.metrics)
    try:
        assert requests.get(base + "/healthz", timeout=5).status_code == 503  # not started yet
        plugin.start()
        kubelet.wait_for(RES)
        r = requests.get(base + "/healthz", timeout=5)
        assert r.status_code == 200 and r.text == "ok"
        wedge.set()
        assert _wait(lambda: not plugin.liveness(monitor_stall_s=0.1)[0], timeout=10)  # the loop enters the wedged call
        ok, why = plugin.liveness(monitor_stall_s=0.1)
        assert not ok and "monitor loop stalled" in why
        release.set()
        wedge.clear()
        assert _wait(lambda: plugin.liveness(monitor_stall_s=0.1)[0], timeout=5)
        # the kubelet goes away for good: the socket vanishes and registration keeps failing
        kubelet.stop()
        os.unlink(plugin.cfg.socket_path)
        assert _wait(lambda: plugin._register_failing_since is not None, timeout=20)
        ok, why = plugin.liveness(register_fail_s=0.0)
        assert not ok and "re-registration" in why
        assert plugin.liveness(register_fail_s=3600)[0]  # within the grace period it is still alive
    finally:
        release.set()
        srv.shutdown()
        plugin.stop()
        kubelet.stop()
    assert not plugin.liveness()[0]  # stopped
