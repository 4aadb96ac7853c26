"""Idle-time link re-probe vs pod admission (VERDICT r2 "next" #1, ADVICE r2 plugin.py:441).

The kubelet never retries a failed device-plugin Allocate: the pod is rejected (UnexpectedAdmissionError)
and ends Failed.  So a re-probe must never make Allocate fail.  The contract tested here:
  * the plugin marks its node ``<prefix>/probing: <deadline>`` before probing and clears it after;
  * the extender's /filter rejects a marked node, /sort scores it 0 and /bind refuses it;
  * an Allocate that still arrives mid-probe cancels the probe and succeeds once the links are free;
  * the fake kubelet treats any Allocate / GetPreferredAllocation error as the real one does.
"""
import threading
import time

import grpc
import numpy as np
import pytest

from gpu_topology_on_k8s_amd.deviceplugin import AdmissionError, DevicePluginServer, PluginConfig, placeholder_dev_tree
from gpu_topology_on_k8s_amd.deviceplugin import proto as pb
from gpu_topology_on_k8s_amd.extender import ExtenderConfig, TopologyExtender
from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations, probing_until
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.sim import SimCluster
from gpu_topology_on_k8s_amd.topology import fixtures as fx

C = Contract()


def _probed(t, base=70.0, degrade=None):
    n = t.n
    bw = np.full((n, n), base)
    np.fill_diagonal(bw, np.nan)
    if degrade:
        i, j, f = degrade
        bw[i, j] = bw[j, i] = base * f
    t.set_measured_bw(bw, {"method": "p2p_read_lds", "preset": "quick", "ts": 1700000000})
    return t


class BlockingProbe:
    """A re-probe that runs until released or cancelled (the child-process probe is killed on cancel)."""

    def __init__(self, result):
        self.result = result
        self.started = threading.Event()
        self.release = threading.Event()
        self.cancelled = False

    def __call__(self, cancel=None):
        self.started.set()
        while not self.release.is_set():
            if cancel is not None and cancel.is_set():
                self.cancelled = True
                return None
            time.sleep(0.01)
        return self.result


class Ctx:
    def abort(self, code, msg):
        raise RuntimeError(code, msg)


def _wait(cond, timeout=10.0):
    t0 = time.time()
    while not cond():
        assert time.time() - t0 < timeout, "condition not reached"
        time.sleep(0.01)


def test_probe_marks_node_and_allocate_mid_probe_cancels_it(tmp_path):
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    t = _probed(fx.f7_mi355x(n=4))
    probe = BlockingProbe(_probed(fx.f7_mi355x(n=4), degrade=(0, 1, 0.3)))
    plug = DevicePluginServer(t, PluginConfig(node_name="n1", dev_root=placeholder_dev_tree(str(tmp_path), t), probe_settle_s=0.0),
                              api=api, reprobe_fn=probe)
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("r", plug.reprobe()))
    th.start()
    assert probe.started.wait(5)
    until = probing_until(api.get_node("n1")["metadata"]["annotations"], C)
    assert until > time.time() + 200  # marked for the probe's whole budget
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=["1", "2"])
    t0 = time.time()
    resp = plug.Allocate(req, Ctx())  # never refused: the probe yields
    assert len(resp.container_responses) == 1 and time.time() - t0 < 5
    th.join(5)
    assert out["r"] is False and probe.cancelled and plug.republished == 0
    assert "probing" not in "".join(api.get_node("n1")["metadata"]["annotations"])  # mark cleared
    text = plug.metrics.exposition().decode()
    assert 'gtk_plugin_reprobes_total{result="cancelled"} 1.0' in text
    assert 'gtk_plugin_allocations_total{outcome="probe_yield"} 1.0' in text


def test_probe_that_cannot_be_cancelled_still_admits_after_the_yield_bound(tmp_path):
    """A reprobe_fn without a cancel argument: Allocate waits at most probe_yield_s, then proceeds; the
    measurement is dropped (the Allocate cancelled it, and devices were claimed meanwhile)."""
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    t = _probed(fx.f7_mi355x(n=2))
    done = threading.Event()

    def slow():
        done.wait(3)
        return _probed(fx.f7_mi355x(n=2), degrade=(0, 1, 0.3))

    plug = DevicePluginServer(t, PluginConfig(node_name="n1", dev_root=placeholder_dev_tree(str(tmp_path), t), probe_settle_s=0.0,
                                              probe_yield_s=0.3), api=api, reprobe_fn=slow)
    api.create_pod(make_pod("p", gpus=1, node="n1"))  # bound around the extender; arrives mid-probe below
    api.delete_pod("default", "p")
    th = threading.Thread(target=plug.reprobe)
    th.start()
    _wait(lambda: plug._probing)
    api.create_pod(make_pod("p", gpus=1, node="n1"))
    req = pb.AllocateRequest()
    req.container_requests.add(devices_ids=["1"])
    t0 = time.time()
    assert len(plug.Allocate(req, Ctx()).container_responses) == 1
    assert 0.25 <= time.time() - t0 < 2.5
    done.set()
    th.join(5)
    assert plug.republished == 0
    assert 'gtk_plugin_reprobes_total{result="cancelled"} 1.0' in plug.metrics.exposition().decode()


def test_probe_aborts_when_a_bind_lands_in_the_settle_window():
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    calls = []
    plug = DevicePluginServer(_probed(fx.f7_mi355x(n=4)), PluginConfig(node_name="n1", probe_settle_s=0.2), api=api,
                              reprobe_fn=lambda: calls.append(1))
    th = threading.Thread(target=lambda: api.create_pod(make_pod("late", gpus=2, node="n1")) if not time.sleep(0.05) else None)
    th.start()
    assert plug.reprobe() is False and calls == []
    th.join()
    assert probing_until(api.get_node("n1")["metadata"]["annotations"], C) == 0.0
    assert 'gtk_plugin_reprobes_total{result="busy"} 1.0' in plug.metrics.exposition().decode()


def test_extender_skips_a_marked_node_until_the_deadline():
    now = [1000.0]
    api = FakeAPIServer()
    ann = encode_node_annotations(fx.f7_mi355x(), C)
    for n in ("a", "b"):
        api.create_node(make_node(n, annotations=ann, capacity={C.resource_name: "8"}))
    ext = TopologyExtender(api, ExtenderConfig(resync_s=0.0), clock=lambda: now[0])
    pod = api.create_pod(make_pod("p", gpus=8))
    api.patch_node("a", annotations={C.probing_key: "1300"})
    ok, failed = ext.filter(pod, ["a", "b"])
    assert ok == ["b"] and "link probe in progress" in failed["a"]
    assert dict(ext.prioritize(pod, ["a", "b"])) == {"a": 0, "b": 10}
    with pytest.raises(Exception, match="link probe in progress"):
        ext.bind("default", "p", "", "a")
    now[0] = 1301.0  # a crashed plugin's mark expires on its own
    ok, _ = ext.filter(pod, ["a", "b"])
    assert ok == ["a", "b"]
    assert "gtk_extender_probing_skips_total 3.0" in ext.metrics.exposition().decode()


def test_sim_pod_submitted_mid_probe_goes_elsewhere_or_waits_never_rejected():
    """Two idle 8-GPU nodes; node a starts a re-probe.  An 8-GPU pod submitted mid-probe lands on b; a
    second one finds no feasible node and stays Pending (not Failed); once the probe ends it is placed
    on a and admitted.  The kubelets reject nothing."""
    nodes = {"a": fx.f7_mi355x(link_gbps=76.5), "b": fx.f7_mi355x(link_gbps=76.5)}
    with SimCluster(nodes) as c:
        pa = c.nodes["a"].plugin
        probe = BlockingProbe(None)
        pa.reprobe_fn = probe
        pa.cfg.probe_settle_s = 0.0
        th = threading.Thread(target=pa.reprobe)
        th.start()
        assert probe.started.wait(5)
        c.submit("first", 8)
        r = c.schedule_pending()[0]
        assert r.error == "" and r.node == "b" and len(r.allocated) == 8
        c.submit("second", 8)
        r = c.schedule_pending()[0]
        assert r.node is None and c.api.get_pod("default", "second")["status"]["phase"] == "Pending"
        probe.release.set()
        th.join(5)
        r = c.schedule_pending()[0]
        assert r.error == "" and r.node == "a" and len(r.allocated) == 8
        assert c.assignment("second").assigned is True
        assert c.nodes["a"].kubelet.rejected == [] and c.nodes["b"].kubelet.rejected == []


def test_sim_pod_bound_around_the_extender_mid_probe_is_admitted():
    """The residual race: a pod reaches the kubelet while the probe runs (bound before the mark was
    seen, or by another scheduler).  Allocate cancels the probe and the pod runs."""
    with SimCluster({"a": fx.f7_mi355x(link_gbps=76.5)}) as c:
        pa = c.nodes["a"].plugin
        probe = BlockingProbe(None)
        pa.reprobe_fn = probe
        pa.cfg.probe_settle_s = 0.0
        th = threading.Thread(target=pa.reprobe)
        th.start()
        assert probe.started.wait(5)
        pod = c.api.create_pod(make_pod("direct", gpus=8, node="a"))
        c.nodes["a"].kubelet.admit(pod, c.resource)
        th.join(5)
        assert probe.cancelled and c.api.get_pod("default", "direct")["status"]["phase"] == "Running"
        assert c.assignment("direct").assigned is True and len(c.assignment("direct").group) == 8


def test_fake_kubelet_rejects_for_good_on_an_allocate_error(tmp_path):
    """What the real kubelet does with any Allocate error: the pod is Failed (UnexpectedAdmissionError)."""
    with SimCluster({"a": fx.f7_mi355x(n=2)}) as c:
        plug = c.nodes["a"].plugin

        def broken(request, context):
            context.abort(grpc.StatusCode.UNAVAILABLE, "try later")

        plug.Allocate = broken  # the handler table is built per serve(): re-serve to pick it up
        plug._server.stop(0).wait()
        plug.serve()
        pod = c.api.create_pod(make_pod("x", gpus=1, node="a"))
        with pytest.raises(AdmissionError, match="UnexpectedAdmissionError"):
            c.nodes["a"].kubelet.admit(pod, c.resource)
        st = c.api.get_pod("default", "x")["status"]
        assert st["phase"] == "Failed" and st["reason"] == "UnexpectedAdmissionError"
        assert c.nodes["a"].kubelet.rejected and c.nodes["a"].kubelet.rejected[0][0] == "default/x"


def test_device_ids_that_are_not_indices_are_refused_as_invalid_argument(tmp_path):
    """The kubelet only sends IDs that ListAndWatch advertised; anything else is INVALID_ARGUMENT,
    never an UNKNOWN error out of the handler."""
    t = fx.f7_mi355x(n=4)
    plug = DevicePluginServer(t, PluginConfig(node_name="n1", dev_root=placeholder_dev_tree(str(tmp_path), t)))
    bad = pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=["0", "gpu-1"])])
    with pytest.raises(RuntimeError) as e:
        plug.Allocate(bad, Ctx())
    assert e.value.args[0] == grpc.StatusCode.INVALID_ARGUMENT and "gpu-1" in e.value.args[1]
    pref = pb.PreferredAllocationRequest(container_requests=[pb.ContainerPreferredAllocationRequest(
        available_deviceIDs=["0", "x"], must_include_deviceIDs=[], allocation_size=1)])
    with pytest.raises(RuntimeError) as e:
        plug.GetPreferredAllocation(pref, Ctx())
    assert e.value.args[0] == grpc.StatusCode.INVALID_ARGUMENT
    ok = plug.Allocate(pb.AllocateRequest(container_requests=[pb.ContainerAllocateRequest(devices_ids=["2"])]), Ctx())
    assert ok.container_responses[0].envs["GTK_GPU_GROUP"] == "2"


def test_reprobe_never_overlaps_another_maintenance_operation(tmp_path):
    """A partition switch (deviceplugin/repartition.py) holds ``plugin.maintenance``; a re-probe that
    comes due meanwhile is skipped, not run against GPUs being reconfigured."""
    api = FakeAPIServer()
    api.create_node(make_node("n1"))
    t = _probed(fx.f7_mi355x(n=4))
    probe = BlockingProbe(_probed(fx.f7_mi355x(n=4)))
    probe.release.set()
    plug = DevicePluginServer(t, PluginConfig(node_name="n1", dev_root=placeholder_dev_tree(str(tmp_path), t), probe_settle_s=0.0),
                              api=api, reprobe_fn=probe)
    with plug.maintenance:
        assert plug.reprobe() is False and not probe.started.is_set()
    assert 'gtk_plugin_reprobes_total{result="busy"} 1.0' in plug.metrics.exposition().decode()
    plug.reprobe()
    assert probe.started.is_set()
