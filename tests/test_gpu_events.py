"""GPU event notification (amdsmi) in the device plugin: resets hold a device Unhealthy between the
RAS polls, a finished reset triggers a link re-measurement, VM faults / throttling are recorded.

The native watcher (``_topo.EventWatcher``) runs against the stand-in amdsmi
(``csrc/topo/fake_amdsmi.cpp``), whose events come from a script file."""
import tempfile
import threading
import time

import pytest

from gpu_topology_on_k8s_amd._native import available, binary
from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig
from gpu_topology_on_k8s_amd.deviceplugin.events import GpuEventWatcher
from gpu_topology_on_k8s_amd.deviceplugin.health import HealthMonitor
from gpu_topology_on_k8s_amd.k8s import FakeAPIServer
from gpu_topology_on_k8s_amd.k8s.objects import make_node
from gpu_topology_on_k8s_amd.topology import fixtures as fx

PRE, POST, VMFAULT, THERMAL = 3, 4, 1, 2  # amdsmi_evt_notification_type_t


def _fake_lib():
    if not available("_topo"):
        pytest.skip("_topo not built")
    try:
        return str(binary("libfake_amdsmi.so"))
    except Exception:
        pytest.skip("fake_amdsmi not built")


def test_native_watcher_delivers_masked_events_by_pci_address(tmp_path, monkeypatch):
    from gpu_topology_on_k8s_amd._native import load

    script = tmp_path / "events"
    script.write_text(f"2 {PRE} reset requested\n5 {VMFAULT} addr 0x1000\n")
    monkeypatch.setenv("FAKE_AMDSMI_EVENTS_FILE", str(script))
    monkeypatch.setenv("FAKE_AMDSMI_GPUS", "8")
    w = load("_topo").EventWatcher(_fake_lib(), ["GPU_PRE_RESET", "GPU_POST_RESET"])  # VM faults not subscribed
    try:
        assert len(w.bdfs) == 8
        ev = w.poll(200, 16)
        assert ev == [(w.bdfs[2], "GPU_PRE_RESET", "reset requested")]
        t0 = time.monotonic()
        assert w.poll(100, 16) == []  # nothing new: returns after the timeout
        assert time.monotonic() - t0 >= 0.09
        with open(script, "a") as f:  # appended while watching: next poll
            f.write(f"2 {POST} done\n")
        assert w.poll(200, 16) == [(w.bdfs[2], "GPU_POST_RESET", "done")]
    finally:
        w.close()
    with pytest.raises(Exception):
        load("_topo").EventWatcher(_fake_lib(), ["NOT_AN_EVENT"])


def _plugin(tmp_health=None, reprobe_fn=None, **cfg):
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    d = tempfile.mkdtemp(prefix="gtke", dir="/tmp")
    topo = fx.f7_mi355x()
    plug = DevicePluginServer(topo, PluginConfig(node_name="n1", socket_dir=d, **cfg), api=api,
                              health_fn=tmp_health, reprobe_fn=reprobe_fn)
    return plug, api


def test_reset_holds_device_unhealthy_until_post_reset():
    state = {"topo": fx.f7_mi355x()}
    plug, api = _plugin(HealthMonitor(fx.f7_mi355x(), lambda: state["topo"]), health_interval=0.05)
    plug.start(register=False)
    try:
        plug.gpu_event(3, "GPU_PRE_RESET", "reset")
        assert plug._health[3] is False
        time.sleep(0.3)  # several RAS passes see nothing wrong: the hold wins
        assert plug._health[3] is False
        plug.gpu_event(3, "GPU_POST_RESET", "done")
        deadline = time.monotonic() + 3
        while not plug._health[3] and time.monotonic() < deadline:
            time.sleep(0.05)
        assert plug._health[3] is True
        reasons = [e["reason"] for e in api.events]
        assert "GPUReset" in reasons and "GPUResetDone" in reasons and "GPUUnhealthy" in reasons
    finally:
        plug.stop()


def test_vmfault_and_throttle_are_recorded_not_fatal():
    plug, api = _plugin()
    plug.gpu_event(1, "VMFAULT", "page 0xdead")
    plug.gpu_event(1, "THERMAL_THROTTLE", "hotspot")
    assert plug._health[1] is True
    assert plug.metrics.gpu_events.labels("VMFAULT")._value.get() == 1
    assert {"GPUVMFault", "GPUThermalThrottle"} <= {e["reason"] for e in api.events}


def test_post_reset_triggers_reprobe_when_idle():
    calls = []

    def reprobe():
        calls.append(time.monotonic())
        return None  # no usable topology: nothing republished

    plug, _ = _plugin(reprobe_fn=reprobe, reprobe_interval=0.0)
    plug.node_idle = lambda: True
    plug.event_source = GpuEventWatcher(source=_ListSource([]))
    plug.start(register=False)
    try:
        time.sleep(0.2)
        assert calls == []  # interval 0 = never on a timer
        plug.gpu_event(0, "GPU_POST_RESET", "")
        deadline = time.monotonic() + 3
        while not calls and time.monotonic() < deadline:
            time.sleep(0.05)
        assert len(calls) == 1
    finally:
        plug.stop()


class _ListSource:
    def __init__(self, events):
        self.events = list(events)
        self.closed = False

    def poll(self, timeout_ms, max_events):
        if self.events:
            out, self.events = self.events[:max_events], self.events[max_events:]
            return out
        time.sleep(timeout_ms / 1000.0)
        return []

    def close(self):
        self.closed = True


def test_watcher_thread_maps_bdf_to_device_and_closes():
    plug, _ = _plugin()
    bdf = plug.topology.gpus[6].bdf
    src = _ListSource([(bdf.upper(), "GPU_PRE_RESET", "x"), ("0000:ff:00.0", "VMFAULT", "other node")])
    w = GpuEventWatcher(source=src, poll_ms=20)
    stop = threading.Event()
    th = threading.Thread(target=w.run, args=(plug, stop), daemon=True)
    th.start()
    deadline = time.monotonic() + 3
    while plug._health[6] and time.monotonic() < deadline:
        time.sleep(0.02)
    stop.set()
    th.join(2)
    assert plug._health[6] is False and w.unmatched == 1 and src.closed


def test_daemon_runs_native_watcher_against_fake_amdsmi(tmp_path, monkeypatch):
    """End to end in process: the watcher the daemon opens (GpuEventWatcher.try_open over amdsmi)
    feeds a plugin whose devices were discovered through the same library."""
    from gpu_topology_on_k8s_amd.topology.discovery import discover

    lib = _fake_lib()
    script = tmp_path / "events"
    script.write_text("")
    monkeypatch.setenv("FAKE_AMDSMI_EVENTS_FILE", str(script))
    monkeypatch.setenv("FAKE_AMDSMI_GPUS", "8")
    topo = discover("amdsmi", amdsmi_lib=lib, pci_root=str(tmp_path), node_root=str(tmp_path))
    w = GpuEventWatcher.try_open(lib, poll_ms=50)
    assert w is not None
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    plug = DevicePluginServer(topo, PluginConfig(node_name="n1", socket_dir=tempfile.mkdtemp(prefix="gtke", dir="/tmp")), api=api)
    plug.event_source = w
    plug.start(register=False)
    try:
        with open(script, "a") as f:
            f.write(f"4 {PRE} driver reset\n")
        deadline = time.monotonic() + 3
        while plug._health[4] and time.monotonic() < deadline:
            time.sleep(0.02)
        assert plug._health[4] is False and w.delivered[0][1] == "GPU_PRE_RESET"
    finally:
        plug.stop()
    assert GpuEventWatcher.try_open("/nonexistent/libamd_smi.so") is None
