"""Taking one GPU out of service without draining its node (``<prefix>/cordoned-gpus``, an operator's
node annotation; docs/OPERATIONS.md).  The device plugin holds the named GPUs Unhealthy: the kubelet's
allocatable shrinks, the extender never chooses them, pods already on them keep running, and removing
the annotation puts them back."""
import pytest

from gpu_topology_on_k8s_amd.k8s import Contract
from gpu_topology_on_k8s_amd.k8s.objects import annotations as obj_annotations
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.shares import time_slice

C = Contract()


def _wait(pred, timeout=5.0):
    import time

    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.02)
    return False


def _cordon(c, node, value):
    c.api.patch_node(node, annotations={C.cordon_key: value})
    return c.nodes[node].plugin.poll_node()


def test_a_cordoned_gpu_is_never_chosen_and_its_running_pod_stays():
    t = fx.f7_mi355x()
    t.gpus[5].bdf = "0000:75:00.0"
    with SimCluster({"n": t}) as c:
        c.submit("on-two", 2)
        (r,) = c.schedule_pending()
        held = set(r.allocated)
        kub, res = c.nodes["n"].kubelet, c.resource
        victim = min(held)
        _cordon(c, "n", f"{victim},75:00.0")  # an index and a PCI address without its domain
        assert _wait(lambda: kub.plugins[res].devices[str(victim)] != "Healthy")
        assert _wait(lambda: c.api.get_node("n")["status"]["allocatable"][res] == "6")
        assert set(kub.allocated[res]["default/on-two"]) == {str(i) for i in held}  # still running
        assert c.nodes["n"].plugin.metrics.cordoned._value.get() == 2
        reasons = [e.get("reason") for e in c.api.events]
        assert "GPUCordoned" in reasons
        c.extender.cache.sync_all()
        c.submit("big", 4)
        (r2,) = c.schedule_pending()
        assert r2.node == "n" and not ({victim, 5} & set(r2.allocated)), r2
        c.submit("rest", 2)
        (r3,) = c.schedule_pending()
        assert r3.node is None  # 8 - 2 held - 4 - 2 cordoned: nothing left
        # back in service
        _cordon(c, "n", "")
        assert _wait(lambda: kub.plugins[res].devices[str(victim)] == "Healthy")
        assert "GPUUncordoned" in [e.get("reason") for e in c.api.events]
        c.extender.cache.sync_all()
        c.delete("rest")
        c.submit("rest2", 1)
        (r4,) = c.schedule_pending()
        assert r4.node == "n" and r4.allocated == (5,), r4


def test_a_cordon_names_the_whole_physical_gpu_and_reports_unknown_tokens():
    t = time_slice(fx.f7_mi355x(), 2)  # 16 slices, two per GPU
    with SimCluster({"n": t}) as c:
        plug = c.nodes["n"].plugin
        got, unknown = plug.cordoned_from("3, 0000:ff:00.0, 99, gpu7, ¹")
        assert got == {2, 3} and unknown == ["0000:ff:00.0", "99", "gpu7", "¹"]
        add, drop = plug.apply_cordon("3,99")
        assert add == {2, 3} and not drop
        assert "GPUCordonUnknown" in [e.get("reason") for e in c.api.events]
        assert not plug._health[2] and not plug._health[3]
        # a reset hold outlives an uncordon of the same device
        plug._holds[2] = "GPU reset in progress"
        add, drop = plug.apply_cordon("")
        assert drop == {3} and plug._health[3] and not plug._health[2]


def test_the_daemon_applies_a_cordon_before_it_serves_and_follows_it():
    """The plugin daemon (its own process, against the apiserver over HTTP): a GPU cordoned before it
    starts is never advertised Healthy, and an uncordon is picked up by the periodic node check."""
    import os
    import shutil
    import tempfile

    from gpu_topology_on_k8s_amd.deviceplugin.kubelet import FakeKubelet
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer, serve_http
    from gpu_topology_on_k8s_amd.k8s.objects import make_node
    from test_daemons import _spawn, _stop

    api = FakeAPIServer()
    api.create_node(make_node("worker-1", annotations={C.cordon_key: "2"}))
    srv, url = serve_http(api)
    sockdir = tempfile.mkdtemp(prefix="gtkc", dir="/tmp")
    kubelet = FakeKubelet(sockdir, node_name="worker-1", api=api)
    kubelet.start()
    devroot = os.path.join(sockdir, "dev")
    os.makedirs(devroot)
    p = _spawn(["gpu_topology_on_k8s_amd.deviceplugin", "--discovery", "fake", "--fake-gpus", "4", "--apiserver", url,
                "--node-name", "worker-1", "--socket-dir", sockdir, "--log-level", "WARNING", "--dev-root", devroot,
                "--label-check-interval", "1"])
    try:
        plugin = kubelet.wait_for("amd.com/gpu", timeout=60)
        first = dict(plugin.devices)  # the first ListAndWatch answer
        assert first["2"] == "Unhealthy" and first["0"] == "Healthy", first
        api.patch_node("worker-1", annotations={C.cordon_key: ""})
        assert _wait(lambda: plugin.devices.get("2") == "Healthy", 15)
    finally:
        rc = _stop(p)
        kubelet.stop()
        srv.shutdown()
        shutil.rmtree(sockdir, ignore_errors=True)
    assert rc == 0


def test_a_cordoned_gpu_stays_out_of_service_through_a_reset():
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        plug = c.nodes["n"].plugin
        plug.apply_cordon("3")
        plug.gpu_event(3, "GPU_PRE_RESET")
        plug.gpu_event(3, "GPU_POST_RESET")
        assert plug._health[3] is False and plug._holds[3] == plug.CORDON_HOLD
        plug.gpu_event(4, "GPU_PRE_RESET")  # an uncordoned GPU comes back after its reset
        assert plug._health[4] is False
        plug.gpu_event(4, "GPU_POST_RESET")
        assert plug._health[4] is True
        plug.apply_cordon("")
        assert plug._health[3] is True
        # cordoned while a reset is in progress: the reset's end leaves it cordoned, not Healthy
        plug.gpu_event(5, "GPU_PRE_RESET")
        assert plug.apply_cordon("5")[0] == {5} and plug._holds[5] != plug.CORDON_HOLD
        plug.gpu_event(5, "GPU_POST_RESET")
        assert plug._health[5] is False and plug._holds[5] == plug.CORDON_HOLD
        # uncordoned while a reset is in progress: the reset keeps it out until it ends
        plug.gpu_event(5, "GPU_PRE_RESET")
        assert plug.apply_cordon("") == (set(), set()) and plug._health[5] is False
        plug.gpu_event(5, "GPU_POST_RESET")
        assert plug._health[5] is True and 5 not in plug._holds


def test_a_cordon_outlasts_health_passes_that_find_the_gpu_healthy():
    """The RAS poll reports every GPU healthy; a cordoned one stays out of service through its passes
    and comes back only when the annotation lets it go."""
    with SimCluster({"n": fx.f7_mi355x()}) as c:
        plug = c.nodes["n"].plugin
        kub, res = c.nodes["n"].kubelet, c.resource
        calls = []

        def all_healthy(t):
            calls.append(1)
            return {i: True for i in range(t.n)}

        plug.cfg.health_interval = 0.05
        plug.health_fn = all_healthy
        _cordon(c, "n", "6")
        n0 = len(calls)
        assert _wait(lambda: len(calls) >= n0 + 3)
        assert kub.plugins[res].devices["6"] == "Unhealthy" and not plug._health[6]
        _cordon(c, "n", "")
        assert _wait(lambda: kub.plugins[res].devices["6"] == "Healthy")


def test_any_annotation_text_parses_without_raising():
    """The annotation is free text an operator types: whatever it holds, the plugin names only devices
    it has, whole physical GPUs, and reports the rest."""
    from hypothesis import given, settings
    from hypothesis import strategies as st

    from gpu_topology_on_k8s_amd.deviceplugin.plugin import DevicePluginServer

    t = time_slice(fx.f7_mi355x(), 2)
    for i, g in enumerate(t.gpus):
        g.bdf = f"0000:{0x10 + g.physical:02x}:00.0"
    plug = DevicePluginServer(t)
    token = st.one_of(st.integers(-5, 40).map(str), st.sampled_from([g.bdf for g in t.gpus] + ["14:00.0", "0000:FF:00.0"]),
                      st.text(max_size=8))

    @settings(max_examples=300, deadline=None)
    @given(st.lists(token, max_size=6).map(",".join))
    def check(value):
        got, unknown = plug.cordoned_from(value)
        assert got <= set(range(t.n))
        for i in got:  # whole physical GPUs
            assert {g.index for g in t.gpus if g.physical == t.gpus[i].physical} <= got
        assert all(isinstance(u, str) and u for u in unknown)

    check()
