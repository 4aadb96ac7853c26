"""GPU: node-local device indices reach the right HIP device by PCI address (VERDICT r1 "next" #1).

A fixture topology whose index 3 carries the real GPU's PCI address stands in for "the pod got
GROUP=3 on an 8-GPU node": inside such a pod HIP numbers its only device 0."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def real_bdf():
    from gpu_topology_on_k8s_amd.topology.identity import hip_device_bdfs

    bdfs = hip_device_bdfs()
    assert bdfs and bdfs[0], "no HIP device / PCI address"
    return bdfs[0]


def _fixture_with_real_gpu_at(index, real, n=4):
    from gpu_topology_on_k8s_amd.topology.discovery import fake_topology

    t = fake_topology(n)
    for g in t.gpus:  # addresses no real device has
        g.bdf = f"00ff:{0xe0 + g.index:02x}:1f.7"
    t.gpus[index].bdf = real
    return t


def test_hip_bdf_matches_amdsmi_discovery(real_bdf):
    from gpu_topology_on_k8s_amd.topology.discovery import discover
    from gpu_topology_on_k8s_amd.topology.identity import DeviceMap

    t = discover("auto")
    m = DeviceMap.for_topology(t)
    assert m.by_bdf and m.complete, (real_bdf, [g.bdf for g in t.gpus])
    assert m.hip(m.index(0)) == 0


def test_validate_group_3_runs_on_hip_0(real_bdf, tmp_path):
    t = _fixture_with_real_gpu_at(3, real_bdf)
    path = tmp_path / "node.json"
    path.write_text(t.to_json())
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "validate", "--topology", str(path),
                        "--min-bytes", str(1 << 20), "--max-bytes", str(16 << 20), "--iters", "3", "--warmup", "1"],
                       capture_output=True, text=True, cwd=REPO, timeout=300, env=dict(os.environ, GTK_GPU_GROUP="3"))
    assert p.returncode == 0, p.stderr[-3000:]
    summary = json.loads([l for l in p.stdout.splitlines() if l.startswith('{"summary"')][-1])
    assert summary["devices"] == [0] and summary["wrong"] == 0 and summary["k"] == 1


def test_validate_with_allocate_env_bdfs(real_bdf):
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "validate", "--min-bytes", str(1 << 20),
                        "--max-bytes", str(1 << 20), "--iters", "2", "--warmup", "1"],
                       capture_output=True, text=True, cwd=REPO, timeout=300,
                       env=dict(os.environ, GTK_GPU_GROUP="6", GTK_GPU_BDFS=real_bdf.upper()))
    assert p.returncode == 0, p.stderr[-3000:]
    summary = json.loads([l for l in p.stdout.splitlines() if l.startswith('{"summary"')][-1])
    assert summary["devices"] == [0] and summary["wrong"] == 0


def test_probe_writes_the_mapped_row(real_bdf):
    from gpu_topology_on_k8s_amd.ops.probe import probe_topology

    t = _fixture_with_real_gpu_at(2, real_bdf)
    probe_topology(t, preset="quick")
    assert t.probe["device_map"] == "bdf" and t.probe["devices"] == [2] and t.probe["hip_ordinals"] == [0]
    assert np.isfinite(t.hbm_gbps[2]) and t.hbm_gbps[2] > 500
    assert not np.isfinite(t.hbm_gbps[[0, 1, 3]]).any()


def test_choose_subset_binds_by_bdf(real_bdf):
    from gpu_topology_on_k8s_amd.parallel.allreduce import choose_subset

    t = _fixture_with_real_gpu_at(5, real_bdf, n=8)
    ch = choose_subset(1, topology=t)
    assert ch.devices == [5] and ch.hip_devices == [0] and ch.extra["device_map"]["by_bdf"]


def test_bench_under_hip_visible_devices_keeps_probe():
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3", "--warmup", "1", "--size-mb", "64",
                        "--sweep", "off", "--graph", "off"], capture_output=True, text=True, timeout=600, cwd=REPO, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    cfg = out["config"]
    assert cfg["probed"] is True and "mesh" not in cfg["topology_source"], cfg
    assert cfg["hip_devices"] == [0] and out["link_probe"]["hbm_copy_gbps"][cfg["subset"][0]] > 500


def test_prestart_validation_on_real_node():
    """Flow step 8 on MI355X: kubelet PreStartContainer -> the plugin runs `gtk validate` in a child
    over the allocated device (GROUP -> HIP ordinal by PCI address) and records RCCL's result."""
    from gpu_topology_on_k8s_amd.k8s import Contract
    from gpu_topology_on_k8s_amd.sim import SimCluster
    from gpu_topology_on_k8s_amd.topology.discovery import discover

    t = discover("auto")
    t.node_name = "gpu-node"
    with SimCluster({"gpu-node": t}, prestart_validate=True) as c:
        c.submit("validated", 1)
        r = c.schedule_pending()[0]
        assert r.error == "" and len(r.allocated) == 1
        v = json.loads(c.api.get_pod("default", "validated")["metadata"]["annotations"][Contract().validated_key])
        assert v["k"] == 1 and v["peak_algbw_gbps"] > 100


def test_pod_flow_then_training_on_the_allocated_device():
    """Flow steps 1-7 on the real node, then the workload inside the 'container': the device plugin's
    Allocate envs (GTK_GPU_GROUP/GTK_GPU_BDFS) decide where the MNIST job trains (design.md:239)."""
    from gpu_topology_on_k8s_amd.sim import SimCluster
    from gpu_topology_on_k8s_amd.topology.discovery import discover

    t = discover("auto")
    t.node_name = "gpu-node"
    with SimCluster({"gpu-node": t}) as c:
        c.submit("trainer", 1)
        r = c.schedule_pending()[0]
        assert r.error == "" and len(r.allocated) == 1
        resp = c.nodes["gpu-node"].kubelet.responses["default/trainer"]
        envs = dict(resp.container_responses[0].envs)
    assert envs["GTK_GPU_GROUP"] == str(r.allocated[0]) and envs["GTK_GPU_BDFS"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update({k: envs[k] for k in ("GTK_GPU_GROUP", "GTK_GPU_BDFS")})
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd.models.train", "--model", "mnist-cnn", "--batch", "64",
                        "--steps", "20", "--warmup", "2", "--gemm-tuning", "off"], capture_output=True, text=True, cwd=REPO,
                       timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["devices"] == [r.allocated[0]] and out["images_per_s"] > 0


def test_the_allocated_env_opens_ipc_handles_across_processes():
    """The device plugin hands each container the IPC mode multi-process RCCL needs on these hosts
    (HSA_ENABLE_IPC_MODE_LEGACY=0, the plugin's own setting in the manifests): a process started with
    only the container's value exports a buffer that a second process opens and reads exactly."""
    from gpu_topology_on_k8s_amd.sim import SimCluster
    from gpu_topology_on_k8s_amd.topology.discovery import discover

    t = discover("auto")
    t.node_name = "gpu-node"
    with SimCluster({"gpu-node": t}) as c:
        c.nodes["gpu-node"].plugin.cfg.container_ipc_mode = "0"
        c.submit("ipc", 1)
        r = c.schedule_pending()[0]
        assert r.error == "" and len(r.allocated) == 1
        envs = dict(c.nodes["gpu-node"].kubelet.responses["default/ipc"].container_responses[0].envs)
    assert envs["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "HSA_ENABLE_IPC_MODE_LEGACY")}
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = envs["HSA_ENABLE_IPC_MODE_LEGACY"]
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "ipc", "--bytes", str(64 << 20)], capture_output=True,
                       text=True, timeout=300, cwd=REPO, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stderr[-2000:]
    out = json.loads(lines[-1])
    assert out["ok"] and out["ipc_mode_legacy"] == "0", out
