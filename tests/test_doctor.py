"""``gtk doctor``: node and pod readiness checks, one JSON line each."""
import json
import os
import subprocess
import sys

from gpu_topology_on_k8s_amd.doctor import check_cpu_affinity, check_ipc, check_pod, run_checks
from gpu_topology_on_k8s_amd.topology import fixtures as fx

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _by_name(checks):
    return {c["name"]: c for c in checks}


def test_node_checks_on_a_fake_node():
    c = _by_name(run_checks("fake", 4, env={"HSA_ENABLE_IPC_MODE_LEGACY": "0"}, plugin_dir="/nonexistent"))
    assert c["discovery"]["status"] == "ok" and c["discovery"]["devices"] == 4 and c["discovery"]["link_types"] == ["XGMI"]
    assert c["native"]["status"] == "ok" and c["vgpu-guard"]["status"] == "ok" and c["ipc-mode"]["status"] == "ok"
    assert c["device-plugin-dir"]["status"] == "skip" and c["pod-group"]["status"] == "skip"
    assert check_ipc({})["status"] == "warn"


def test_cpu_affinity_check():
    t = fx.f7_mi355x(n=4)
    for g in t.gpus:
        g.cpu_affinity = "0-7" if g.numa == 0 else "8-15"
    assert check_cpu_affinity(t, allowed=range(16))["status"] == "ok"
    r = check_cpu_affinity(t, allowed=range(8))
    assert r["status"] == "warn" and "[2, 3]" in r["detail"]


def test_pod_checks_from_an_allocate_env():
    """What Allocate put into a container holding half of GPU 1 (time slices): GROUP maps by PCI address,
    the cpuset is usable, and the share needs its CU mask and the guard."""
    env = {"GTK_GPU_GROUP": "1", "GTK_GPU_BDFS": "0000:75:00.0", "GTK_CPUSET": "4-7", "GTK_GPU_FRACTION": "0.5",
           "HSA_CU_MASK": "0:0-127"}
    c = _by_name(check_pod(env, visible_bdfs=["0000:75:00.0"], allowed=range(8)))
    assert c["pod-group"]["status"] == "ok" and c["pod-group"]["hip_devices"] == [0]
    assert c["pod-cpuset"]["status"] == "ok"
    assert c["pod-share"]["status"] == "warn" and "guard" in c["pod-share"]["detail"]
    c = _by_name(check_pod(dict(env, GTK_VGPU_ACTIVE="1"), visible_bdfs=["0000:75:00.0"], allowed=range(8)))
    assert c["pod-share"]["status"] == "ok"
    bare = {k: v for k, v in env.items() if k != "HSA_CU_MASK"}  # the guard cleared it: it masks the queues
    c = _by_name(check_pod(dict(bare, GTK_VGPU_ACTIVE="1"), visible_bdfs=["0000:75:00.0"], allowed=range(8)))
    assert c["pod-share"]["status"] == "ok" and "by the guard" in c["pod-share"]["detail"]
    c = _by_name(check_pod(bare, visible_bdfs=["0000:75:00.0"], allowed=range(8)))
    assert c["pod-share"]["status"] == "warn" and "no HSA_CU_MASK" in c["pod-share"]["detail"]
    c = _by_name(check_pod(env, visible_bdfs=["0000:05:00.0"], allowed=range(100, 108)))
    assert c["pod-group"]["status"] == "fail" and c["pod-cpuset"]["status"] == "warn"


def test_cli_exit_status_and_json_lines():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "doctor", "--discovery", "fake", "--fake-gpus", "2",
                        "--plugin-dir", "/nonexistent"], capture_output=True, text=True, timeout=120, cwd=REPO, env=env)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines[-1]["summary"] and lines[-1]["status"] in ("ok", "warn")
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "doctor", "--discovery", "sysfs", "--dev-root", "/nonexistent"],
                       capture_output=True, text=True, timeout=120, cwd=REPO, env=env)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 1 and lines[-1]["status"] == "fail"  # no /dev/kfd, no GPUs in this container


def test_ipc_cli_reports_a_failed_export_as_json():
    """`gtk ipc` without a usable GPU: one JSON line naming the failed stage, exit 1 (on MI355X it
    reads a peer process's buffer: tests/test_gpu_native.py::test_ipc_read_across_processes)."""
    import torch

    if torch.cuda.is_available():
        return
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "ipc", "--bytes", "1048576"], capture_output=True,
                       text=True, timeout=120, cwd=REPO)
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert p.returncode == 1 and out["ok"] is False and out["stage"].startswith("export")
