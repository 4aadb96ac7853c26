"""The two daemons as shipped (``python -m ...deviceplugin`` / ``python -m ...extender``) in subprocesses,
talking to an in-test fake kubelet (gRPC, unix socket) and the fake apiserver over HTTP."""
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time

import pytest
import requests

from gpu_topology_on_k8s_amd.deviceplugin import FakeKubelet
from gpu_topology_on_k8s_amd.k8s import Contract, FakeAPIServer, serve_http
from gpu_topology_on_k8s_amd.k8s.annotations import encode_node_annotations
from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod
from gpu_topology_on_k8s_amd.topology import fixtures as fx

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _wait(pred, timeout=30.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.05)
    return False


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


def test_device_plugin_daemon_registers_and_publishes():
    api = FakeAPIServer()
    api.create_node(make_node("worker-1"))
    srv, url = serve_http(api)
    sockdir = tempfile.mkdtemp(prefix="gtkd", dir="/tmp")
    kubelet = FakeKubelet(sockdir, node_name="worker-1", api=api)
    kubelet.start()
    mport = _free_port()
    devroot = os.path.join(sockdir, "dev")  # a kind node: no ROCm device nodes at all
    os.makedirs(devroot)
    p = _spawn(["gpu_topology_on_k8s_amd.deviceplugin", "--discovery", "fake", "--fake-gpus", "4", "--apiserver", url,
                "--node-name", "worker-1", "--socket-dir", sockdir, "--resource-name", "aliyun.com/gpu", "--log-level", "WARNING",
                "--dev-root", devroot, "--metrics-port", str(mport), "--metrics-host", "127.0.0.1"])
    try:
        plugin = kubelet.wait_for("aliyun.com/gpu", timeout=60)
        assert sorted(plugin.devices) == ["0", "1", "2", "3"]
        node = api.get_node("worker-1")
        assert "GPU_XGMI_0_1" in node["metadata"]["annotations"]
        assert node["status"]["capacity"]["aliyun.com/gpu"] == "4"
        pod = api.create_pod(make_pod("p", gpus=2, node="worker-1", resource="aliyun.com/gpu"))
        resp = kubelet.admit(pod, "aliyun.com/gpu")  # the fake kubelet rejects host paths that do not exist
        c = resp.container_responses[0]
        assert list(c.devices) == []  # --discovery fake => stub DeviceSpecs: envs + annotations only (BASELINE config 1)
        assert c.envs["GTK_GPU_GROUP"] and len(c.envs["GTK_GPU_BDFS"].split(",")) == 2
        scrape = lambda: requests.get(f"http://127.0.0.1:{mport}/metrics", timeout=5).text  # noqa: E731
        assert _wait(lambda: "gtk_plugin_registrations_total 1.0" in scrape(), 10)  # counted once Register returns
        assert 'gtk_plugin_allocations_total{outcome="ok"} 1.0' in scrape()
    finally:
        rc = _stop(p)
        kubelet.stop()
        srv.shutdown()
        shutil.rmtree(sockdir, ignore_errors=True)
    assert rc == 0, p.stdout.read() if p.stdout else ""


def test_extender_daemon_serves_the_reference_endpoint():
    api = FakeAPIServer()
    c = Contract()
    api.create_node(make_node("n1", annotations=encode_node_annotations(fx.f7_mi355x(), c), capacity={c.resource_name: "8"}))
    srv, url = serve_http(api)
    port = _free_port()
    p = _spawn(["gpu_topology_on_k8s_amd.extender", "--apiserver", url, "--port", str(port), "--host", "127.0.0.1",
                "--log-level", "WARNING"])
    base = f"http://127.0.0.1:{port}/gputopology-scheduler"
    try:
        def up():
            try:
                return requests.get(base + "/healthz", timeout=1).ok
            except requests.RequestException:
                return False

        assert _wait(up, 60), "extender did not come up"
        pod = api.create_pod(make_pod("train", gpus=4))
        hp = requests.post(base + "/sort", json={"Pod": pod, "NodeNames": ["n1"]}, timeout=10).json()
        assert hp[0]["Host"] == "n1" and hp[0]["Score"] >= 1
        br = requests.post(base + "/bind", json={"PodName": "train", "PodNamespace": "default",
                                                 "PodUID": pod["metadata"]["uid"], "Node": "n1"}, timeout=10).json()
        assert br["Error"] == "" and len(br["Devices"]) == 4
        assert api.get_pod("default", "train")["spec"]["nodeName"] == "n1"
        assert "gtk_extender_binds_total" in requests.get(base + "/metrics", timeout=5).text
    finally:
        _stop(p)
        srv.shutdown()


def test_both_daemons_config4_through_shipped_processes():
    """BASELINE config 4 with the shipped entry points only: the device-plugin daemon (fake 8-GPU node,
    stub DeviceSpecs) publishes to the apiserver and registers with the kubelet; the extender daemon
    (LIST+WATCH informer) answers /filter, /sort and /bind; two 4-GPU pods land on disjoint NUMA halves
    and the kubelet admits both."""
    api = FakeAPIServer()
    api.create_node(make_node("worker-1"))
    srv, url = serve_http(api)
    sockdir = tempfile.mkdtemp(prefix="gtkd", dir="/tmp")
    devroot = os.path.join(sockdir, "dev")
    os.makedirs(devroot)
    kubelet = FakeKubelet(sockdir, node_name="worker-1", api=api)
    kubelet.start()
    port = _free_port()
    plug = _spawn(["gpu_topology_on_k8s_amd.deviceplugin", "--discovery", "fake", "--fake-gpus", "8", "--apiserver", url,
                   "--node-name", "worker-1", "--socket-dir", sockdir, "--dev-root", devroot, "--log-level", "WARNING"])
    ext = _spawn(["gpu_topology_on_k8s_amd.extender", "--apiserver", url, "--port", str(port), "--log-level", "WARNING"])
    base = f"http://127.0.0.1:{port}/gputopology-scheduler"
    try:
        kubelet.wait_for("amd.com/gpu", timeout=60)

        def up():
            try:
                return requests.get(base + "/healthz", timeout=1).ok
            except requests.RequestException:
                return False

        assert _wait(up, 60), "extender did not come up"
        assert _wait(lambda: requests.post(base + "/filter", json={"Pod": make_pod("probe", gpus=8), "NodeNames": ["worker-1"]},
                                           timeout=5).json()["NodeNames"] == ["worker-1"], 30)  # informer saw the topology
        got = []
        for name in ("a", "b"):
            pod = api.create_pod(make_pod(name, gpus=4))
            names = requests.post(base + "/filter", json={"Pod": pod, "NodeNames": ["worker-1"]}, timeout=10).json()["NodeNames"]
            hp = requests.post(base + "/sort", json={"Pod": pod, "NodeNames": names}, timeout=10).json()
            br = requests.post(base + "/bind", json={"PodName": name, "PodNamespace": "default", "PodUID": pod["metadata"]["uid"],
                                                     "Node": hp[0]["Host"]}, timeout=10).json()
            assert br["Error"] == "", br
            kubelet.admit(api.get_pod("default", name), "amd.com/gpu")
            got.append(set(br["Devices"]))
        assert {frozenset(g) for g in got} == {frozenset(range(4)), frozenset(range(4, 8))}
        for name in ("a", "b"):
            ann = api.get_pod("default", name)["metadata"]["annotations"]
            assert ann["ALIYUN_COM_GPU_ASSIGNED"] == "true" and ann[Contract().cpuset_key]
        assert any(e["reason"] == "GPUTopologyBound" for e in api.events)
    finally:
        _stop(ext)
        rc = _stop(plug)
        kubelet.stop()
        srv.shutdown()
        shutil.rmtree(sockdir, ignore_errors=True)
    assert rc == 0


def test_device_plugin_daemon_time_slices():
    """A node labelled ``gputopology.amd.com/time-slices=4`` (no flag): the kubelet sees 8 devices of the
    slice resource (and no whole GPUs), the node annotation carries the slices, and a 2-slice pod gets
    one GPU's device nodes with GTK_GPU_FRACTION=0.5."""
    from gpu_topology_on_k8s_amd.k8s.annotations import decode_node_annotations
    from gpu_topology_on_k8s_amd.topology.shares import slices_per_gpu

    api = FakeAPIServer()
    api.create_node(make_node("worker-1", labels={"gputopology.amd.com/time-slices": "4"}))  # the operator's per-node choice
    srv, url = serve_http(api)
    sockdir = tempfile.mkdtemp(prefix="gtkd", dir="/tmp")
    kubelet = FakeKubelet(sockdir, node_name="worker-1", api=api)
    kubelet.start()
    devroot = os.path.join(sockdir, "dev")
    os.makedirs(devroot)
    guard_dir = os.path.join(sockdir, "vgpu")
    p = _spawn(["gpu_topology_on_k8s_amd.deviceplugin", "--discovery", "fake", "--fake-gpus", "2", "--label-check-interval", "2",
                "--apiserver", url, "--node-name", "worker-1", "--socket-dir", sockdir, "--dev-root", devroot,
                "--share-guard-dir", guard_dir, "--log-level", "WARNING"])
    try:
        plugin = kubelet.wait_for("amd.com/gpu-slice", timeout=60)
        assert sorted(plugin.devices, key=int) == [str(i) for i in range(8)] and "amd.com/gpu" not in kubelet.plugins
        ann = api.get_node("worker-1")["metadata"]["annotations"]
        topo = decode_node_annotations(ann, Contract())
        assert topo.n == 8 and slices_per_gpu(topo) == 4 and ann[Contract().active_slices_key] == "4"
        pod = api.create_pod(make_pod("half", gpus=2, node="worker-1", resource="amd.com/gpu-slice"))
        c = kubelet.admit(pod, "amd.com/gpu-slice").container_responses[0]
        assert c.envs["GTK_GPU_FRACTION"] == "0.5" and len(c.envs["GTK_GPU_GROUP"].split(",")) == 1
        # the daemon's default --share-guard env: the vGPU guard mounted and preloaded (host paths exist)
        m = {x.container_path: x.host_path for x in c.mounts}
        assert c.envs["LD_PRELOAD"] == "/usr/local/lib/gtk-vgpu/libgtk_vgpu.so"
        assert m["/usr/local/lib/gtk-vgpu/libgtk_vgpu.so"] == os.path.join(guard_dir, "libgtk_vgpu.so")
        assert all(os.path.exists(h) for h in m.values())
        # the operator relabels the node: the plugin waits while a pod holds devices, then exits for a
        # restart (EX_TEMPFAIL) with the new slicing
        api.patch_node("worker-1", labels={"gputopology.amd.com/time-slices": "2"})
        with pytest.raises(subprocess.TimeoutExpired):
            p.wait(timeout=6)
        api.delete_pod("default", "half")
        assert p.wait(timeout=60) == 75
        # the old layout stays published until the restart: the extender is told to keep away
        assert Contract().probing_key in api.get_node("worker-1")["metadata"]["annotations"]
        return
    finally:
        rc = _stop(p)
        kubelet.stop()
        srv.shutdown()
        shutil.rmtree(sockdir, ignore_errors=True)
    assert rc == 0, p.stdout.read() if p.stdout else ""


def _pki(d):
    """A CA, a server certificate for 127.0.0.1 and a client certificate, with the openssl CLI."""
    def run(*args):
        subprocess.run(["openssl", *args], check=True, capture_output=True, cwd=d)

    run("req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", "ca.key", "-out", "ca.crt", "-days", "2", "-subj", "/CN=test-ca")
    with open(os.path.join(d, "san.cnf"), "w") as f:
        f.write("subjectAltName=IP:127.0.0.1\n")
    for name, ext in (("server", ["-extfile", "san.cnf"]), ("client", [])):
        run("req", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{name}.key", "-out", f"{name}.csr", "-subj", f"/CN={name}")
        run("x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial", "-out", f"{name}.crt",
            "-days", "2", *ext)
    return {n: os.path.join(d, n) for n in ("ca.crt", "server.crt", "server.key", "client.crt", "client.key")}


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI not available")
def test_extender_daemon_mutual_tls():
    """--tls-cert/--tls-key/--client-ca: the extender serves HTTPS and only answers callers whose
    certificate the CA signed (kube-scheduler's extender tlsConfig), so /bind may leave loopback."""
    api = FakeAPIServer()
    srv, url = serve_http(api)
    d = tempfile.mkdtemp(prefix="gtkpki", dir="/tmp")
    pki = _pki(d)
    port = _free_port()
    ext = _spawn(["gpu_topology_on_k8s_amd.extender", "--apiserver", url, "--port", str(port), "--log-level", "WARNING",
                  "--tls-cert", pki["server.crt"], "--tls-key", pki["server.key"], "--client-ca", pki["ca.crt"]])
    base = f"https://127.0.0.1:{port}/gputopology-scheduler"
    try:
        def up():
            try:
                return requests.get(base + "/healthz", timeout=1, verify=pki["ca.crt"],
                                    cert=(pki["client.crt"], pki["client.key"])).ok
            except requests.RequestException:
                return False

        assert _wait(up, 60), "extender did not come up over TLS"
        with pytest.raises(requests.exceptions.ConnectionError):  # no client certificate: handshake refused / closed
            requests.get(base + "/healthz", timeout=5, verify=pki["ca.crt"])
        with pytest.raises(requests.RequestException):
            requests.post(base.replace("https", "http") + "/bind", json={}, timeout=5)  # plain HTTP is not served
    finally:
        rc = _stop(ext)
        srv.shutdown()
        shutil.rmtree(d, ignore_errors=True)
    assert rc == 0, ext.stdout.read() if ext.stdout else ""


def test_restart_on_a_busy_node_keeps_the_published_slicing():
    """a plugin restarted (crash, rollout) after the operator relabelled the node keeps the
    slice count it last published while any pod holds a device; an idle node switches at once."""
    from gpu_topology_on_k8s_amd.deviceplugin.__main__ import startup_time_slices
    from gpu_topology_on_k8s_amd.k8s import PodAssignment

    c = Contract()
    api = FakeAPIServer()
    api.create_node(make_node("n", labels={c.time_slices_label: "2"}, annotations={c.active_slices_key: "4"}))
    api.create_pod(make_pod("busy", gpus=2, node="n", resource=c.slice_resource,
                            annotations=PodAssignment([4, 5], True, 1).to_annotations()))
    s, why = startup_time_slices(api, "n", c, 1)
    assert s == 4 and "keeping 4" in why
    api.delete_pod("default", "busy")
    s, why = startup_time_slices(api, "n", c, 1)
    assert s == 2 and "4 -> 2" in why
    api.create_node(make_node("fresh", labels={c.time_slices_label: "4"}))  # first start: nothing published
    assert startup_time_slices(api, "fresh", c, 1) == (4, "")
    assert startup_time_slices(None, "", c, 3) == (3, "")


def test_plugin_soak_harness_on_a_fake_node():
    """bench/plugin_soak.py (run on MI355X with re-probes: profiles/r03_soak/): the shipped daemon under
    pod churn, here on a fake 2-GPU node sliced in two, with concurrent partial-GPU pods."""
    import json

    p = subprocess.run([sys.executable, os.path.join(REPO, "bench", "plugin_soak.py"), "--discovery", "fake", "--probe", "off",
                        "--seconds", "4", "--max-idle", "0.3", "--hold", "0.2", "--time-slices", "2"],
                       capture_output=True, text=True, timeout=180, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{"discovery"')][-1])
    assert out["rejected"] == 0 and out["admitted"] >= 3 and out["guarded"] >= 1 and out["daemon_exit"] == 0
