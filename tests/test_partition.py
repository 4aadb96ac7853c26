"""Hardware partition control (topology/partition.py, deviceplugin/repartition.py) on the stand-in
amdsmi (csrc/topo/fake_amdsmi.cpp): MI300-class rules, no TPX, NPS4 only together with CPX, and a
memory mode that waits for a driver reload.  No GPU box runs a setter: switching partitions there
would change a shared machine (and needs root).  ``tests/test_gpu_native.py`` reads the real modes."""
import os
import shutil
import signal
import subprocess
import sys
import tempfile

import pytest

from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer, serve_http
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.topology.discovery import discover
from gpu_topology_on_k8s_amd.topology.partition import PartitionError, apply_partition, partition_info, plan_steps

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _spawn(args):
    env = dict(os.environ, PYTHONPATH=REPO)
    return subprocess.Popen([sys.executable, "-m", *args], cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            text=True)


def _stop(p):
    if p.poll() is None:
        p.send_signal(signal.SIGTERM)
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return p.returncode


def _wait_for(pred, timeout=60.0):
    import time

    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if pred():
                return True
        except Exception:  # noqa: BLE001 - not there yet
            pass
        time.sleep(0.1)
    return False


def _lib():
    from gpu_topology_on_k8s_amd._native import binary

    try:
        return str(binary("libfake_amdsmi.so"))
    except Exception:
        pytest.skip("fake_amdsmi not built")


@pytest.fixture
def node(monkeypatch, tmp_path):
    """A 2-package fake node in SPX/NPS1 whose partition state lives in a file."""
    state = tmp_path / "amdsmi_state"
    state.write_text("1 NPS1 -\n")
    for k in ("FAKE_AMDSMI_PARTITIONS", "FAKE_AMDSMI_HIP_ORDER", "FAKE_AMDSMI_DOWN", "FAKE_AMDSMI_SET_STATUS"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("FAKE_AMDSMI_GPUS", "2")
    monkeypatch.setenv("FAKE_AMDSMI_STATE", str(state))
    lib = _lib()
    monkeypatch.setenv("GTK_AMDSMI_LIB", lib)
    return {"lib": lib, "state": state, "tmp": tmp_path}


def _discover(node):
    return discover("amdsmi", amdsmi_lib=node["lib"], pci_root=str(node["tmp"]), node_root=str(node["tmp"]))


def test_plan_orders_steps_by_what_the_modes_allow():
    assert plan_steps("SPX", "NPS1", "CPX", "NPS4") == [("compute", "CPX"), ("memory", "NPS4")]  # finer: compute first
    assert plan_steps("CPX", "NPS4", "SPX", "NPS1") == [("memory", "NPS1"), ("compute", "SPX")]  # coarser: memory first
    assert plan_steps("CPX", "NPS1", "CPX", None) == []
    assert plan_steps("SPX", "NPS1", None, "NPS1") == []


def test_info_reports_the_offered_modes(node):
    info = partition_info()
    assert [p["bdf"] for p in info] == ["0000:05:00.0", "0000:15:00.0"]
    assert all(p["compute"] == "SPX" and p["memory"] == "NPS1" and p["xcps"] == 1 for p in info)
    assert info[0]["compute_modes"] == ["SPX", "DPX", "QPX", "CPX"] and info[0]["memory_modes"] == ["NPS1", "NPS4"]


def test_spx_to_cpx_and_back_through_a_driver_reload(node):
    r = apply_partition("CPX")
    assert r["ok"] and [s["set"] for s in r["steps"]] == ["compute"] and all(p["compute"] == "CPX" for p in r["after"])
    t = _discover(node)
    assert t.n == 16 and all(g.partition == "CPX" for g in t.gpus) and t.physical.tolist() == [i // 8 for i in range(16)]
    # NPS4 (CPX only) needs the driver reload to take effect
    r = apply_partition("CPX", "NPS4")
    assert not r["ok"] and r["reload_required"] and "reload" in r["reason"]
    r = apply_partition("CPX", "NPS4", reload_driver=True)
    assert r["ok"] and r["reloaded"] and all(p["memory"] == "NPS4" for p in r["after"])
    # back to SPX: NPS1 must come first (SPX refuses NPS4), so memory -> reload -> compute
    r = apply_partition("SPX", "NPS1", reload_driver=True)
    assert r["ok"], r["reason"]
    assert [s["set"] for s in r["steps"]] == ["memory", "driver-reload", "compute"]
    assert _discover(node).n == 2


def test_refusals_are_reported_not_retried(node, monkeypatch):
    with pytest.raises(PartitionError, match="offers compute modes"):
        apply_partition("TPX")  # valid name, not offered by this part
    with pytest.raises(PartitionError, match="unknown compute partition"):
        apply_partition("XPX")
    monkeypatch.setenv("FAKE_AMDSMI_SET_STATUS", "10")
    r = apply_partition("CPX")
    assert not r["ok"] and "permission denied" in r["reason"] and len(r["steps"]) == 1
    assert _discover(node).n == 2


def test_repartition_pass_marks_the_node_and_records_the_outcome(node):
    from gpu_topology_on_k8s_amd.deviceplugin.repartition import repartition

    c = Contract()
    api = FakeAPIServer()
    api.create_node(make_node("w", labels={c.partition_request_label: "CPX"}))
    marks = []

    def idle():
        marks.append((api.get_node("w")["metadata"].get("annotations") or {}).get(c.probing_key))
        return True

    assert repartition(api, "w", c, idle, settle_s=0.01) == ("ok", "SPX/NPS1 -> CPX/-")
    assert marks[-1]  # the extender was told to keep away while the switch ran
    # ... and still is: the published layout is stale until the restarted plugin publishes the new one
    assert c.probing_key in api.get_node("w")["metadata"]["annotations"]
    api.patch_node("w", annotations={c.probing_key: None})  # what the restarted plugin does
    assert any(e["reason"] == "GPUPartitionChanged" for e in api.events)
    assert repartition(api, "w", c, idle)[0] == "same"
    # a busy node waits; a refused switch is recorded once and not retried until the label changes
    api.patch_node("w", labels={c.partition_request_label: "QPX"})
    assert repartition(api, "w", c, lambda: False)[0] == "busy"
    os.environ["FAKE_AMDSMI_SET_STATUS"] = "10"
    try:
        out, msg = repartition(api, "w", c, idle, settle_s=0)
        assert out == "failed" and "permission" in msg
        assert api.get_node("w")["metadata"]["annotations"][c.partition_failed_key].startswith("QPX/-: ")
        assert repartition(api, "w", c, idle, settle_s=0)[0] == "skipped"
    finally:
        del os.environ["FAKE_AMDSMI_SET_STATUS"]
    assert c.probing_key not in api.get_node("w")["metadata"]["annotations"]  # a refusal clears the mark
    api.patch_node("w", labels={c.partition_request_label: "DPX"})
    assert repartition(api, "w", c, idle, settle_s=0)[0] == "ok"
    assert c.partition_failed_key not in api.get_node("w")["metadata"]["annotations"]
    api.patch_node("w", labels={c.partition_request_label: "bogus"})
    assert repartition(api, "w", c, idle)[0] == "invalid"
    # a failure mark left from an earlier request goes once the node is in the requested mode (an operator
    # switched it by hand): "already there" clears it
    api.patch_node("w", labels={c.partition_request_label: "DPX"},
                   annotations={c.partition_failed_key: "DPX/-: an earlier refusal"})
    assert repartition(api, "w", c, idle)[0] == "same"
    assert c.partition_failed_key not in api.get_node("w")["metadata"]["annotations"]


def test_repartition_without_packages_is_not_already_there(node, monkeypatch):
    """amdsmi reporting no package (driver down, no GPU visible) is not "already in the mode": the
    pass says so, records nothing on the node and asks again next time."""
    from gpu_topology_on_k8s_amd.deviceplugin import repartition as rp

    c = Contract()
    api = FakeAPIServer()
    api.create_node(make_node("w", labels={c.partition_request_label: "CPX"}))
    monkeypatch.setattr(rp, "partition_info", lambda lib=None: [])
    out, msg = rp.repartition(api, "w", c, lambda: True, settle_s=0)
    assert out == "unavailable" and "no GPU packages" in msg
    ann = api.get_node("w")["metadata"].get("annotations") or {}
    assert c.partition_failed_key not in ann and c.probing_key not in ann


def test_device_plugin_daemon_repartitions_on_the_node_label(node):
    """The shipped daemon with --partition-control on: a node labelled CPX registers 16 XCPs of a
    2-package node at start-up; relabelled SPX while a pod holds an XCP, the plugin waits, and once
    the pod is gone it switches and exits 75 for a restart."""
    from gpu_topology_on_k8s_amd.deviceplugin import FakeKubelet

    c = Contract()
    api = FakeAPIServer()
    api.create_node(make_node("worker-1", labels={c.partition_request_label: "CPX"}))
    srv, url = serve_http(api)
    sockdir = tempfile.mkdtemp(prefix="gtkp", dir="/tmp")
    kubelet = FakeKubelet(sockdir, node_name="worker-1", api=api)
    kubelet.start()
    devroot = os.path.join(sockdir, "dev")
    os.makedirs(devroot)
    p = _spawn(["gpu_topology_on_k8s_amd.deviceplugin", "--discovery", "amdsmi", "--partition-control", "on",
                "--label-check-interval", "1", "--probe-settle-seconds", "0.2", "--gpu-events", "off", "--device-specs", "stub",
                "--apiserver", url, "--node-name", "worker-1", "--socket-dir", sockdir, "--dev-root", devroot,
                "--log-level", "WARNING"])
    try:
        plugin = kubelet.wait_for("amd.com/gpu", timeout=60)
        assert len(plugin.devices) == 16
        node_md = api.get_node("worker-1")["metadata"]
        assert node_md["labels"][c.label_partition] == "CPX" and c.probing_key not in node_md["annotations"]
        pod = api.create_pod(make_pod("x", gpus=1, node="worker-1"))
        kubelet.admit(pod, "amd.com/gpu")
        api.patch_node("worker-1", labels={c.partition_request_label: "SPX"})
        with pytest.raises(subprocess.TimeoutExpired):
            p.wait(timeout=5)
        assert node["state"].read_text().split()[0] == "8"
        api.delete_pod("default", "x")
        assert p.wait(timeout=60) == 75
        assert node["state"].read_text().split()[0] == "1"
        assert c.probing_key in api.get_node("worker-1")["metadata"]["annotations"]  # until the restart publishes SPX
        p = _spawn(["gpu_topology_on_k8s_amd.deviceplugin", "--discovery", "amdsmi", "--partition-control", "on",
                    "--gpu-events", "off", "--device-specs", "stub", "--apiserver", url, "--node-name", "worker-1",
                    "--socket-dir", sockdir, "--dev-root", devroot, "--log-level", "WARNING"])
        assert _wait_for(lambda: len(kubelet.plugins.get("amd.com/gpu").devices) == 2 if "amd.com/gpu" in kubelet.plugins else False)
        md = api.get_node("worker-1")["metadata"]
        assert md["labels"][c.label_partition] == "SPX" and c.probing_key not in md["annotations"]
        assert [e["reason"] for e in api.events if "Partition" in e["reason"]] == ["GPUPartitionChanged"] * 2
    finally:
        _stop(p)
        kubelet.stop()
        srv.shutdown()
        shutil.rmtree(sockdir, ignore_errors=True)


def test_partition_cli_show_on_the_fake_node(node):
    out = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "partition", "show"], capture_output=True, text=True,
                         timeout=120, cwd=REPO, env=dict(os.environ))
    assert out.returncode == 0, out.stderr
    assert '"compute": "SPX"' in out.stdout and "CPX" in out.stdout
    out = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "partition", "set", "--compute", "CPX"],
                         capture_output=True, text=True, timeout=120, cwd=REPO, env=dict(os.environ))
    assert out.returncode == 2 and "--yes" in out.stderr  # changing a node's hardware is never implicit
    out = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "partition", "set", "--compute", "CPX", "--yes"],
                         capture_output=True, text=True, timeout=120, cwd=REPO, env=dict(os.environ))
    assert out.returncode == 0, out.stderr + out.stdout
    assert node["state"].read_text().split()[0] == "8"


def test_manifests_with_partition_control_mount_sys_writable():
    import yaml

    from gpu_topology_on_k8s_amd.config import render_manifests

    def plugin(docs):
        ds = next(d for d in docs if d["kind"] == "DaemonSet" and d["metadata"]["name"] == "amd-gpu-topology-device-plugin")
        return ds["spec"]["template"]["spec"]["containers"][0]

    off = plugin(list(yaml.safe_load_all(render_manifests())))
    on = plugin(list(yaml.safe_load_all(render_manifests(partition_control=True))))
    assert "--partition-control=on" not in off["command"] and "--partition-control=on" in on["command"]
    sys_mount = lambda c: next(m for m in c["volumeMounts"] if m["name"] == "sys")  # noqa: E731
    assert sys_mount(off)["readOnly"] is True and sys_mount(on)["readOnly"] is False


def test_partitions_and_time_slices_are_not_stacked(node):
    """A time-sliced node refuses an XCP partition request (recorded, no hardware touched); a
    partitioned node started with --time-slices advertises its XCPs unsliced instead of crashing."""
    from gpu_topology_on_k8s_amd.deviceplugin.repartition import repartition

    c = Contract()
    api = FakeAPIServer()
    api.create_node(make_node("w", labels={c.partition_request_label: "CPX", c.time_slices_label: "4"}))
    out, msg = repartition(api, "w", c, lambda: True, settle_s=0, time_slices=4)
    assert out == "failed" and "time-sliced" in msg and node["state"].read_text().split()[0] == "1"
    assert api.get_node("w")["metadata"]["annotations"][c.partition_failed_key].startswith("CPX/-: ")
    assert repartition(api, "w", c, lambda: True, time_slices=4)[0] == "skipped"

    from gpu_topology_on_k8s_amd.deviceplugin import FakeKubelet

    node["state"].write_text("8 NPS1 -\n")  # the node is CPX already
    srv, url = serve_http(api)
    sockdir = tempfile.mkdtemp(prefix="gtkq", dir="/tmp")
    kubelet = FakeKubelet(sockdir, node_name="w", api=api)
    kubelet.start()
    p = _spawn(["gpu_topology_on_k8s_amd.deviceplugin", "--discovery", "amdsmi", "--gpu-events", "off", "--device-specs", "stub",
                "--apiserver", url, "--node-name", "w", "--socket-dir", sockdir, "--dev-root", sockdir, "--log-level", "ERROR",
                "--label-check-interval", "1"])
    try:
        plug = kubelet.wait_for("amd.com/gpu", timeout=60)  # the XCPs, as whole devices of their own
        assert len(plug.devices) == 16 and "amd.com/gpu-slice" not in kubelet.plugins
        # several label checks later the plugin is still serving: the label's count it cannot apply
        # on a partitioned node is not a layout change (exit-75 restart loop)
        import time

        time.sleep(4.5)
        assert p.poll() is None, p.stdout.read() if p.poll() is not None else ""
        from gpu_topology_on_k8s_amd.k8s.annotations import probing_until

        assert probing_until(api.get_node("w")["metadata"].get("annotations") or {}, c) < time.time()
    finally:
        _stop(p)
        kubelet.stop()
        srv.shutdown()
        shutil.rmtree(sockdir, ignore_errors=True)


class _Ctx:
    def abort(self, code, msg):
        raise RuntimeError(code, msg)


def _held_plugin(tmp_path):
    from gpu_topology_on_k8s_amd.deviceplugin import DevicePluginServer, PluginConfig, placeholder_dev_tree
    from gpu_topology_on_k8s_amd.topology import fixtures as fx

    api = FakeAPIServer()
    api.create_node(make_node("w", labels={Contract().partition_request_label: "CPX"}))
    t = fx.f7_mi355x(n=2)
    plug = DevicePluginServer(t, PluginConfig(node_name="w", dev_root=placeholder_dev_tree(str(tmp_path), t)), api=api)
    return api, plug


def _alloc_req(*ids):
    from gpu_topology_on_k8s_amd.deviceplugin import proto as pb

    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=[str(i) for i in ids])
    return req


def test_allocate_during_the_settle_window_abandons_the_switch(node, tmp_path):
    """ADVICE r3 (repartition.py:100): an Allocate that arrives while a switch is pending (a bind
    that outlived the settle window, or a pod that bypassed the extender) is held, makes the node
    busy, and then proceeds on the unchanged layout; no amdsmi step runs."""
    import threading
    import time

    from gpu_topology_on_k8s_amd.deviceplugin.repartition import repartition

    api, plug = _held_plugin(tmp_path)
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", repartition(
        api, "w", Contract(), lambda: True, settle_s=0.6, hold=plug.allocation_hold)))
    th.start()
    t0 = time.time()
    while plug._hold is None:
        assert time.time() - t0 < 5
        time.sleep(0.01)
    resp = plug.Allocate(_alloc_req(1), _Ctx())  # waits for the pass to give up, then succeeds
    th.join(5)
    assert len(resp.container_responses) == 1
    assert out["r"][0] == "busy"
    assert node["state"].read_text().split()[0] == "1"  # still SPX: amdsmi never ran
    assert Contract().probing_key not in (api.get_node("w")["metadata"].get("annotations") or {})


def test_allocate_held_across_a_switch_is_refused_not_given_stale_devices(node, tmp_path, monkeypatch):
    """An Allocate that arrives once the amdsmi steps run cannot stop them: it waits for the switch and
    is refused (UNAVAILABLE), since its device IDs name the old layout."""
    import threading
    import time

    import grpc

    from gpu_topology_on_k8s_amd.deviceplugin import repartition as rp

    api, plug = _held_plugin(tmp_path)
    started = threading.Event()
    real = rp.apply_partition

    def slow_apply(*a, **kw):
        started.set()
        time.sleep(0.5)
        return real(*a, **kw)

    monkeypatch.setattr(rp, "apply_partition", slow_apply)
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", rp.repartition(
        api, "w", Contract(), lambda: True, settle_s=0, hold=plug.allocation_hold)))
    th.start()
    assert started.wait(5)
    with pytest.raises(RuntimeError) as ei:
        plug.Allocate(_alloc_req(0), _Ctx())
    th.join(5)
    assert out["r"][0] == "ok"
    assert ei.value.args[0] == grpc.StatusCode.UNAVAILABLE and "repartitioned" in ei.value.args[1]
    assert 'gtk_plugin_allocations_total{outcome="switch_wait"} 1.0' in plug.metrics.exposition().decode()


def test_driver_reload_is_held_back_when_the_node_stops_being_idle(node):
    """The last idle check sits right before the amdgpu reload (the most disruptive step)."""
    r = apply_partition("CPX")
    assert r["ok"]
    r = apply_partition("CPX", "NPS4", reload_driver=True, before_reload=lambda: False)
    assert not r["ok"] and r["reload_required"] and "held back" in r["reason"]
    assert not any(s["set"] == "driver-reload" for s in r["steps"])


def test_allocate_held_while_a_reload_is_held_back_proceeds(node, tmp_path, monkeypatch):
    """ADVICE r4 (repartition.py:121): a memory mode set but pending its driver reload changes no
    device; when the reload is held back for the very Allocate that arrived, that Allocate must
    proceed on the (unchanged) layout instead of being refused as stale."""
    import threading
    import time

    from gpu_topology_on_k8s_amd.deviceplugin import repartition as rp

    assert apply_partition("CPX")["ok"]  # CPX/NPS1: the request below is a memory-only change
    api, plug = _held_plugin(tmp_path)
    c = Contract()
    api.patch_node("w", labels={c.partition_request_label: "CPX", c.memory_partition_request_label: "NPS4"})
    real = rp.apply_partition
    started = threading.Event()

    def apply_when_contended(*a, **kw):
        started.set()
        t0 = time.time()
        while not plug._hold.contended():  # the Allocate below is waiting on the hold
            assert time.time() - t0 < 5
            time.sleep(0.01)
        return real(*a, **kw)

    monkeypatch.setattr(rp, "apply_partition", apply_when_contended)
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", rp.repartition(
        api, "w", c, lambda: True, settle_s=0, reload_driver=True, hold=plug.allocation_hold)))
    th.start()
    assert started.wait(5)
    resp = plug.Allocate(_alloc_req(1), _Ctx())  # waits for the switch, then is served: nothing changed
    th.join(5)
    assert len(resp.container_responses) == 1
    assert out["r"][0] == "failed" and "held back" in out["r"][1]
    assert not plug._stale_layout
    # ... and the node is not left marked: nothing to republish
    assert c.probing_key not in (api.get_node("w")["metadata"].get("annotations") or {})


def test_a_partial_switch_is_reported_as_a_layout_change(node, tmp_path, monkeypatch):
    """A compute step that took before a later step failed changed the exposed devices: the pass says
    ``partial`` (the daemon restarts for it, like after ``ok``), held Allocates are refused, and the
    node stays marked until the restarted plugin publishes the new layout."""
    from gpu_topology_on_k8s_amd.deviceplugin import repartition as rp

    api, plug = _held_plugin(tmp_path)
    monkeypatch.setattr(rp, "apply_partition", lambda *a, **kw: {
        "ok": False, "layout_changed": True, "reason": "memory partition NPS4: fake refusal",
        "steps": [{"set": "compute", "mode": "CPX", "packages": [{"bdf": "x", "status": "ok"}]}]})
    outcome, msg = rp.repartition(api, "w", Contract(), lambda: True, settle_s=0, hold=plug.allocation_hold)
    assert outcome == "partial" and "partly applied" in msg
    assert plug._stale_layout
    assert Contract().probing_key in (api.get_node("w")["metadata"].get("annotations") or {})


def test_apply_partition_reports_whether_the_layout_changed(node):
    r = apply_partition("CPX")
    assert r["ok"] and r["layout_changed"]
    r = apply_partition("CPX", "NPS4", reload_driver=False)  # pending a reload: no device changed yet
    assert not r["ok"] and r["reload_required"] and not r["layout_changed"]
    r = apply_partition("CPX", "NPS4", reload_driver=True)
    assert r["ok"] and r["reloaded"] and r["layout_changed"]
