#!/usr/bin/env python3
"""Soak of the device-plugin daemon on a real node: pod churn against idle-time link re-probes.

The shipped daemon (``python -m gpu_topology_on_k8s_amd.deviceplugin``) runs against an in-process
fake apiserver and kubelet.  With ``--probe quick`` it measures the links in a child process at
start-up and again whenever the node has been idle for ``--reprobe-interval`` seconds.  Pods are
created, admitted through the kubelet's gRPC Allocate, held for a moment and deleted, with random idle
gaps between them.  So re-probes start while the node is idle, and the next pod's Allocate often
arrives mid-probe and has to cancel it (plugin.reprobe: the probe child is killed, Allocate waits
for the links and proceeds).

Reported: pods admitted and rejected (the real kubelet never retries a failed Allocate, so this must
be 0), Allocate latency (p50 / p99 / max, including any probe yield), re-probe outcomes, and the
daemon's RSS and open file descriptors over the run (a leak shows up as steady growth).

    python bench/plugin_soak.py --seconds 150 --out profiles/r03_soak/soak.json        # MI355X
    python bench/plugin_soak.py --discovery fake --seconds 20                          # CPU harness check
"""
from __future__ import annotations

import argparse
import json
import os
import random
import shutil
import signal
import socket
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _proc_stats(pid: int) -> dict:
    """RSS (MiB) and open fds of the daemon (children excluded: the probe child comes and goes)."""
    try:
        with open(f"/proc/{pid}/status") as f:
            rss = next(int(ln.split()[1]) for ln in f if ln.startswith("VmRSS:")) / 1024
        fds = len(os.listdir(f"/proc/{pid}/fd"))
        return {"rss_mib": round(rss, 1), "fds": fds}
    except (OSError, StopIteration):
        return {"rss_mib": None, "fds": None}


def _metrics(port: int) -> dict:
    import requests

    out = {}
    try:
        for ln in requests.get(f"http://127.0.0.1:{port}/metrics", timeout=5).text.splitlines():
            if ln.startswith(("gtk_plugin_reprobes_total", "gtk_plugin_allocations_total")):
                k, v = ln.rsplit(" ", 1)
                out[k] = float(v)
    except Exception as e:  # noqa: BLE001 - reported in the row
        out["error"] = str(e)[:100]
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--discovery", default="auto", choices=["auto", "amdsmi", "sysfs", "fake"])
    ap.add_argument("--probe", default="quick", choices=["off", "quick", "full"])
    ap.add_argument("--reprobe-interval", type=float, default=4.0)
    ap.add_argument("--max-idle", type=float, default=8.0, help="longest idle gap between pods (s)")
    ap.add_argument("--hold", type=float, default=0.5, help="longest time a pod holds its device (s)")
    ap.add_argument("--time-slices", type=int, default=1,
                    help="S > 1: the node advertises amd.com/gpu-slice; pods take 1..S slices, several at once, "
                         "and partial-GPU pods get the vGPU guard mounted")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from gpu_topology_on_k8s_amd.deviceplugin import AdmissionError, FakeKubelet
    from gpu_topology_on_k8s_amd.k8s import FakeAPIServer, serve_http
    from gpu_topology_on_k8s_amd.k8s.objects import make_node, make_pod

    rng = random.Random(a.seed)
    api = FakeAPIServer()
    api.create_node(make_node("soak-node"))
    srv, url = serve_http(api)
    sockdir = tempfile.mkdtemp(prefix="gtks", dir="/tmp")
    kubelet = FakeKubelet(sockdir, node_name="soak-node", api=api)
    kubelet.start()
    mport = _free_port()
    args = [sys.executable, "-m", "gpu_topology_on_k8s_amd.deviceplugin", "--discovery", a.discovery, "--probe", a.probe,
            "--reprobe-interval", str(a.reprobe_interval), "--probe-settle-seconds", "0.3", "--probe-yield-seconds", "20",
            "--health-interval", "2", "--apiserver", url, "--node-name", "soak-node", "--socket-dir", sockdir,
            "--metrics-port", str(mport), "--metrics-host", "127.0.0.1", "--log-level", "WARNING"]
    if a.discovery == "fake":
        args += ["--fake-gpus", "2", "--device-specs", "stub", "--dev-root", sockdir]
    resource = "amd.com/gpu"
    if a.time_slices > 1:
        resource = "amd.com/gpu-slice"
        args += ["--time-slices", str(a.time_slices), "--share-guard", "env", "--share-guard-dir", os.path.join(sockdir, "vgpu")]
    log_path = os.path.join(sockdir, "daemon.log")
    logf = open(log_path, "w")
    daemon = subprocess.Popen(args, cwd=REPO, env=dict(os.environ, PYTHONPATH=REPO), stdout=logf, stderr=subprocess.STDOUT)
    lat, rejected, admitted, guarded, samples = [], 0, 0, 0, []
    rc = None
    try:
        plugin = kubelet.wait_for(resource, timeout=300)
        devs = sorted(plugin.devices, key=int)
        t0 = time.time()
        samples.append({"t": 0.0, **_proc_stats(daemon.pid), **_metrics(mport)})
        print(json.dumps({"registered": devs, **samples[-1]}), flush=True)
        i, last = 0, t0
        live: list = []  # (name, slices) of pods holding devices

        def finish(name):
            kubelet.release(api.get_pod("default", name))  # the container ends: its devices go back
            api.delete_pod("default", name)

        while time.time() - t0 < a.seconds:
            if not live:
                time.sleep(rng.uniform(0.0, a.max_idle))  # idle: a re-probe may start now
            want = 1 if a.time_slices <= 1 else rng.randint(1, a.time_slices)
            free = len(kubelet.available(resource))
            if want > free:  # full: the oldest pod ends first
                finish(live.pop(0)[0])
                continue
            pod = api.create_pod(make_pod(f"p{i}", gpus=want, node="soak-node", resource=resource))
            ts = time.perf_counter()
            try:
                resp = kubelet.admit(pod, resource)
                admitted += 1
                envs = resp.container_responses[0].envs
                guarded += int("LD_PRELOAD" in envs)
                live.append((f"p{i}", want))
            except AdmissionError as e:
                rejected += 1
                print(json.dumps({"rejected": f"p{i}", "error": str(e)[:200]}), flush=True)
                api.delete_pod("default", f"p{i}")
            lat.append((time.perf_counter() - ts) * 1e3)
            time.sleep(rng.uniform(0.0, a.hold))
            while live and (a.time_slices <= 1 or rng.random() < 0.5):
                finish(live.pop(0)[0])
            i += 1
            if time.time() - last >= 10:
                last = time.time()
                samples.append({"t": round(last - t0, 1), "pods": i, **_proc_stats(daemon.pid), **_metrics(mport)})
                print(json.dumps(samples[-1]), flush=True)
        for name, _ in live:
            finish(name)
        samples.append({"t": round(time.time() - t0, 1), "pods": i, **_proc_stats(daemon.pid), **_metrics(mport)})
    finally:
        if daemon.poll() is None:
            daemon.send_signal(signal.SIGTERM)
            try:
                rc = daemon.wait(timeout=60)
            except subprocess.TimeoutExpired:
                daemon.kill()
                rc = daemon.wait()
        else:
            rc = daemon.returncode
        logf.close()
        kubelet.stop()
        srv.shutdown()
    with open(log_path) as f:
        tail = f.read()[-3000:]
    shutil.rmtree(sockdir, ignore_errors=True)
    last = samples[-1] if samples else {}
    def label(k: str) -> str:  # gtk_plugin_x_total{outcome="ok"} -> ok
        return k.split('"')[1] if '"' in k else k

    reprobes = {label(k): int(v) for k, v in last.items() if k.startswith("gtk_plugin_reprobes_total{")}
    allocs = {label(k): int(v) for k, v in last.items() if k.startswith("gtk_plugin_allocations_total{")}
    q = sorted(lat)
    out = {
        "discovery": a.discovery, "probe": a.probe, "time_slices": a.time_slices, "seconds": a.seconds, "pods": len(lat),
        "admitted": admitted, "guarded": guarded,
        "rejected": rejected, "allocate_ms": {"p50": round(statistics.median(q), 2) if q else None,
                                              "p99": round(q[int(0.99 * (len(q) - 1))], 2) if q else None,
                                              "max": round(q[-1], 2) if q else None},
        "reprobes": reprobes, "allocations": allocs,
        "rss_mib": [samples[0].get("rss_mib"), last.get("rss_mib")] if samples else None,
        "fds": [samples[0].get("fds"), last.get("fds")] if samples else None,
        "daemon_exit": rc, "samples": samples,
    }
    print(json.dumps({k: v for k, v in out.items() if k != "samples"}), flush=True)
    if rc != 0:
        print(tail, file=sys.stderr)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0 if rc == 0 and rejected == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
