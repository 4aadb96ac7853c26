"""Scheduler config generators, deploy manifests and the operator CLI."""
import json
import subprocess
import sys

import yaml

from gpu_topology_on_k8s_amd.config import legacy_policy, render_manifests, scheduler_configuration


def test_legacy_policy_matches_reference():
    """design.md:92-113, field for field."""
    p = legacy_policy("aliyun.com/gpu")
    assert p["kind"] == "Policy" and p["apiVersion"] == "v1"
    (e,) = p["extenders"]
    assert e == {
        "urlPrefix": "http://127.0.0.1:32743/gputopology-scheduler",
        "PrioritizeVerb": "sort",
        "bindVerb": "bind",
        "enableHttps": False,
        "nodeCacheCapable": True,
        "managedResources": [{"name": "aliyun.com/gpu", "ignoredByScheduler": False}],
        "ignorable": False,
    }
    assert "filterVerb" not in e  # design.md:117: no filter in the reference


def test_scheduler_configuration():
    c = scheduler_configuration("amd.com/gpu", extra_resources=["aliyun.com/gpu"])
    assert c["apiVersion"] == "kubescheduler.config.k8s.io/v1"
    e = c["extenders"][0]
    assert e["prioritizeVerb"] == "sort" and e["bindVerb"] == "bind" and e["filterVerb"] == "filter"
    assert [m["name"] for m in e["managedResources"]] == ["amd.com/gpu", "amd.com/gpu-slice", "aliyun.com/gpu"]


def test_manifests_are_valid_yaml():
    docs = list(yaml.safe_load_all(render_manifests()))
    kinds = [d["kind"] for d in docs]
    assert kinds == ["ServiceAccount", "ServiceAccount", "ClusterRole", "ClusterRoleBinding", "ValidatingAdmissionPolicy",
                     "ValidatingAdmissionPolicyBinding", "ClusterRole", "ClusterRoleBinding", "Role", "RoleBinding",
                     "DaemonSet", "DaemonSet", "ConfigMap"]
    ds, ext_ds = [d for d in docs if d["kind"] == "DaemonSet"]
    assert ext_ds["spec"]["template"]["spec"]["nodeSelector"] == {"node-role.kubernetes.io/control-plane": ""}
    ext = ext_ds["spec"]["template"]["spec"]["containers"][0]
    assert "--host=127.0.0.1" in ext["command"] and "ports" not in ext  # /bind is never exposed off-node
    assert "--ledger-store=lease" in ext["command"]
    c = ds["spec"]["template"]["spec"]["containers"][0]
    assert "gpu_topology_on_k8s_amd.deviceplugin" in c["command"]
    assert {"name": "device-plugins", "mountPath": "/var/lib/kubelet/device-plugins"} in c["volumeMounts"]
    cm = docs[-1]
    assert yaml.safe_load(cm["data"]["scheduler-config.yaml"])["kind"] == "KubeSchedulerConfiguration"


def _cli(*args):
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", *args], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    return p.stdout


def test_cli_topo_select_config():
    out = _cli("topo", "--discovery", "fake", "--fake-gpus", "8", "--output", "json")
    assert json.loads(out)["gpus"][7]["index"] == 7
    ann = json.loads(_cli("topo", "--discovery", "fake", "--fake-gpus", "2", "--output", "annotations"))
    assert ann["GPU_XGMI_0_1"] == "xGMI 1 hop"
    sel = json.loads(_cli("select", "--discovery", "fake", "--fake-gpus", "8", "-k", "4", "--used", "0", "--worst"))
    assert sel["ids"] == [4, 5, 6, 7] and sel["worst"]["score"] < sel["score"]
    g = json.loads(_cli("select", "--discovery", "fake", "--fake-gpus", "8", "-k", "2", "--policy", "gaia"))
    assert len(g["ids"]) == 2
    assert json.loads(_cli("config", "policy"))["kind"] == "Policy"
    fr = json.loads(_cli("select", "--discovery", "fake", "--fake-gpus", "4", "--time-slices", "4", "--fraction", "0.25", "--used", "8,9"))
    assert fr["gpu"] == 2 and fr["ids"] == [10] and fr["share"] == 0.25 and fr["hsa_cu_mask"] == "0:128-191"
    p = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "select", "--discovery", "fake", "--fake-gpus", "4",
                        "--fraction", "0.5"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "time-sliced" in p.stderr


def test_cli_select_explain_on_a_degraded_link(tmp_path):
    """``gtk select --explain``: the chosen, worst and kubelet-default subsets with their terms; with link
    0-1 at 60 % the default (0, 1) is predicted 1 / 0.6 slower than the choice, by link terms."""
    from gpu_topology_on_k8s_amd.topology import fixtures as fx

    f = tmp_path / "t.json"
    f.write_text(fx.f7_degraded(((0, 1, 0.6),)).to_json())
    out = json.loads(_cli("select", "--topology", str(f), "-k", "2", "--explain"))
    ex = out["explain"]
    assert ex["chosen"]["ids"] == out["ids"] and ex["default"]["ids"] == [0, 1] and ex["worst"]["ids"] == out["worst"]["ids"]
    assert ex["vs_default"]["link_terms_separate"] and abs(ex["vs_default"]["predicted_gain"] - 1 / 0.6) < 1e-3


def test_manifests_time_slices():
    from gpu_topology_on_k8s_amd.config import render_manifests

    docs = list(yaml.safe_load_all(render_manifests(time_slices=4)))
    ds = [d for d in docs if d and d["kind"] == "DaemonSet" and "device-plugin" in d["metadata"]["name"]][0]
    assert "--time-slices=4" in ds["spec"]["template"]["spec"]["containers"][0]["command"]
    assert "--time-slices" not in render_manifests()


def test_scheduler_config_mutual_tls():
    from gpu_topology_on_k8s_amd.config import scheduler_configuration

    ext = scheduler_configuration(tls_dir="/etc/gtk/tls")["extenders"][0]
    assert ext["enableHTTPS"] is True and ext["urlPrefix"].startswith("https://127.0.0.1:32743")
    assert ext["tlsConfig"] == {"certFile": "/etc/gtk/tls/tls.crt", "keyFile": "/etc/gtk/tls/tls.key", "caFile": "/etc/gtk/tls/ca.crt"}
    assert scheduler_configuration()["extenders"][0]["enableHTTPS"] is False


def test_cli_sim():
    lines = [json.loads(l) for l in _cli("sim", "--nodes", "1", "--pods", "4,4").splitlines()]
    assert {tuple(l["devices"]) for l in lines} == {(0, 1, 2, 3), (4, 5, 6, 7)}


def test_committed_deploy_files_are_current():
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent / "deploy"
    assert (root / "gpu-topology.yaml").read_text() == render_manifests()
    from gpu_topology_on_k8s_amd.config import render_kind

    for name, text in render_kind().items():
        assert (root / "kind" / name).read_text() == text, name


def test_kind_manifests_config1():
    from gpu_topology_on_k8s_amd.config import render_kind

    files = render_kind()
    docs = list(yaml.safe_load_all(files["gpu-topology-kind.yaml"]))
    ds = [d for d in docs if d["kind"] == "DaemonSet" and d["metadata"]["name"] == "amd-gpu-topology-device-plugin"][0]
    c = ds["spec"]["template"]["spec"]["containers"][0]
    assert "--device-specs=stub" in c["command"] and "--discovery=fake" in c["command"] and "--fake-gpus=2" in c["command"]
    assert {v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]} == {"device-plugins", "pod-resources"}
    kc = yaml.safe_load(files["kind-config.yaml"])
    assert [n["role"] for n in kc["nodes"]] == ["control-plane", "worker"]
    assert yaml.safe_load(files["pod-1gpu.yaml"])["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "1"


def test_console_scripts_resolve():
    """setup.cfg console scripts (gtk, gtk-device-plugin, gtk-extender) point at real callables."""
    import configparser
    import importlib
    import os

    cfg = configparser.ConfigParser()
    cfg.read(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "setup.cfg"))
    lines = [l.strip() for l in cfg["options.entry_points"]["console_scripts"].splitlines() if l.strip()]
    assert {l.split("=")[0].strip() for l in lines} == {"gtk", "gtk-device-plugin", "gtk-extender"}
    for l in lines:
        mod, fn = l.split("=")[1].strip().split(":")
        assert callable(getattr(importlib.import_module(mod), fn))
