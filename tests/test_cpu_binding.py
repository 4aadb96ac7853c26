"""Gaia B6 "GPU and CPU core are automatically bound" (paper p.3 §III.A) in the workload: the pod's
GTK_CPUSET (or the rank's own device slice) intersected with the container's allowed CPUs is applied
to every thread and sizes the intra-op pools (VERDICT r2 "next" #4)."""
import json
import os
import subprocess
import sys

from gpu_topology_on_k8s_amd.topology.cpus import apply_cpuset, bind_workload, format_cpulist, parse_cpulist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_apply_intersects_with_the_allowed_cpus():
    calls = []
    rep = apply_cpuset("0-7,64-71", allowed=set(range(4, 68)), setter=lambda tid, cpus: calls.append(set(cpus)), threads=False)
    assert rep["applied"] and rep["cpus"] == "4-7,64-67" and rep["n"] == 8
    assert calls == [set(range(4, 8)) | set(range(64, 68))]


def test_disjoint_or_empty_cpuset_is_reported_not_applied():
    calls = []
    rep = apply_cpuset("128-191", allowed=set(range(0, 64)), setter=lambda tid, cpus: calls.append(cpus), threads=False)
    assert not rep["applied"] and "disjoint" in rep["reason"] and calls == []
    rep = apply_cpuset("", allowed=set(range(8)), setter=lambda tid, cpus: calls.append(cpus))
    assert not rep["applied"] and rep["reason"] == "no cpuset given" and calls == []


def test_bind_workload_modes():
    seen = []
    kw = {"allowed": set(range(0, 256)), "setter": lambda tid, cpus: seen.append(format_cpulist(cpus)), "threads": False}
    pod = {"GTK_CPUSET": "0-31,128-159"}
    # auto: the pod's cores narrowed to this rank's device slice
    r = bind_workload("auto", "16-31,144-159", env=pod, **kw)
    assert r["applied"] and r["source"] == "GTK_CPUSET&device-slice" and r["cpus"] == "16-31,144-159"
    # auto with a slice outside the pod's cores: the pod's set wins (the kubelet's CPU manager decided)
    r = bind_workload("auto", "64-79", env=pod, **kw)
    assert r["cpus"] == "0-31,128-159" and r["source"] == "GTK_CPUSET"
    # bare node (no pod env): the device slice
    r = bind_workload("auto", "64-79", env={}, **kw)
    assert r["cpus"] == "64-79" and r["source"] == "device-slice"
    assert bind_workload("env", "64-79", env={}, **kw)["applied"] is False
    assert bind_workload("off", "64-79", env=pod, **kw)["applied"] is False


def _child(code, env=None):
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=REPO,
                       env=dict(os.environ, **(env or {})))
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_real_affinity_of_every_thread_and_thread_pools():
    """In a child process (the test runner itself must stay unpinned): a thread started before the
    binding is moved too, and OMP / torch intra-op threads follow the core count."""
    allowed = sorted(os.sched_getaffinity(0))
    want = format_cpulist(allowed[:2])
    code = f"""
import json, os, threading, time, torch
from gpu_topology_on_k8s_amd.topology.cpus import bind_workload
ev = threading.Event(); box = {{}}
def worker():
    ev.wait(); box['aff'] = sorted(os.sched_getaffinity(0))
t = threading.Thread(target=worker); t.start()
rep = bind_workload('env', '')
ev.set(); t.join()
print(json.dumps({{'rep': rep, 'main': sorted(os.sched_getaffinity(0)), 'early_thread': box['aff'],
                  'torch_threads': torch.get_num_threads(), 'omp': os.environ.get('OMP_NUM_THREADS')}}))
"""
    out = _child(code, {"GTK_CPUSET": want})
    assert out["rep"]["applied"] and out["rep"]["cpus"] == want
    assert out["main"] == allowed[:2] and out["early_thread"] == allowed[:2]
    assert out["torch_threads"] == 2 and out["omp"] == "2"


def test_train_entry_point_reports_and_applies_gtk_cpuset():
    allowed = sorted(os.sched_getaffinity(0))
    base = [sys.executable, "-m", "gpu_topology_on_k8s_amd.models.train", "--model", "tiny", "--device", "cpu", "--batch", "1",
            "--seq", "16", "--steps", "1", "--warmup", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    for cpuset, applied in ((format_cpulist(allowed[:1]), True), ("100000", False)):
        p = subprocess.run(base, capture_output=True, text=True, timeout=300, cwd=REPO, env=dict(env, GTK_CPUSET=cpuset))
        assert p.returncode == 0, p.stderr[-2000:]
        rep = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])["cpuset_applied"]
        assert rep["applied"] is applied, rep
        if applied:
            assert parse_cpulist(rep["cpus"]) == set(allowed[:1])
        else:
            assert "disjoint" in rep["reason"]


def test_a_malformed_cpuset_is_reported_not_fatal():
    """GTK_CPUSET comes from a pod annotation a user can edit: a list that does not parse is reported and
    not applied (the rank falls back to its device's own slice), never an exception at start-up."""
    from gpu_topology_on_k8s_amd.topology.cpus import apply_cpuset, bind_workload

    calls = []
    rep = apply_cpuset("0-3,x-7", allowed=set(range(8)), setter=lambda tid, s: calls.append(s))
    assert rep["applied"] is False and "malformed" in rep["reason"] and not calls
    rep = bind_workload("auto", own="4-5", env={"GTK_CPUSET": "garbage"}, allowed=set(range(8)),
                        setter=lambda tid, s: calls.append(s))
    assert rep["applied"] and rep["cpus"] == "4-5" and "malformed" in rep["source"]
