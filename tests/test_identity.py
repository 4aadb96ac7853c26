"""Device identity: topology index <-> PCI BDF <-> HIP ordinal (VERDICT r1 "next" #1).

The visible-BDF lists stand in for ``hipDeviceGetPCIBusId`` so the pod / HIP_VISIBLE_DEVICES cases
run on CPU; ``test_gpu_identity.py`` repeats the key case against the real device."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from gpu_topology_on_k8s_amd.cli import main as cli_main
from gpu_topology_on_k8s_amd.parallel.allreduce import choose_subset, visible_view
from gpu_topology_on_k8s_amd.topology.discovery import fake_topology
from gpu_topology_on_k8s_amd.topology.identity import DeviceMap, normalize_bdf, resolve_group

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _node(n=8):
    t = fake_topology(n)
    for g in t.gpus:  # distinct, realistic addresses: 0000:05:00.0, 0000:15:00.0, ...
        assert normalize_bdf(g.bdf) == g.bdf
    return t


def test_normalize_bdf():
    assert normalize_bdf("0000:05:00.0") == "0000:05:00.0"
    assert normalize_bdf("0000:C5:00.0") == "0000:c5:00.0"
    assert normalize_bdf("c5:00.0") == "0000:c5:00.0"
    assert normalize_bdf("0001:0a:1f.7") == "0001:0a:1f.7"
    assert normalize_bdf("garbage") == "" and normalize_bdf("") == ""


def test_device_map_matches_by_bdf_and_reports_hidden():
    t = _node(8)
    vis = [t.gpus[i].bdf.upper() for i in (4, 5, 6, 7)]  # a pod holding GROUP 4,5,6,7
    m = DeviceMap.for_topology(t, vis)
    assert m.by_bdf and m.complete
    assert [m.hip(i) for i in (4, 5, 6, 7)] == [0, 1, 2, 3]
    assert m.hidden_indices() == [0, 1, 2, 3] and m.visible_indices() == [4, 5, 6, 7]
    with pytest.raises(KeyError, match="not visible"):
        m.hip(0)


def test_device_map_partitions_sharing_one_bdf_match_in_order():
    bdfs = ["0000:05:00.0"] * 4 + ["0000:15:00.0"] * 4  # XCPs reporting their package address
    m = DeviceMap.match(bdfs, ["0000:15:00.0", "0000:15:00.0"])
    assert m.by_bdf and m.hip_of_index == {4: 0, 5: 1}


def test_device_map_without_matches_is_identity_prefix():
    m = DeviceMap.match(["ffff:00:00.0"] * 0 + [f"0000:{i:02x}:00.0" for i in range(4)], ["0000:99:00.0", "0000:98:00.0"])
    assert not m.by_bdf and m.hip_of_index == {0: 0, 1: 1}


def test_resolve_group_paths():
    t = _node(8)
    vis = [t.gpus[i].bdf for i in (6, 2)]  # HIP order inside a pod is PCI order; deliberately shuffled here
    # 1. GTK_GPU_BDFS wins
    assert resolve_group([2, 6], bdfs=[t.gpus[2].bdf, t.gpus[6].bdf], visible_bdfs=vis) == [1, 0]
    # 2. topology file
    assert resolve_group([6, 2], topology=t, visible_bdfs=vis) == [0, 1]
    # 3. exactly |group| visible, no addresses: sorted GROUP -> 0..k-1
    assert resolve_group([6, 2], visible_bdfs=["x", "y"]) == [1, 0]
    # 4. host run with every index present
    assert resolve_group([1, 3], visible_bdfs=["a", "b", "c", "d"]) == [1, 3]
    with pytest.raises(ValueError):
        resolve_group([4, 5, 6], visible_bdfs=["a", "b"])
    with pytest.raises(ValueError, match="not all visible"):
        resolve_group([4], bdfs=["0000:77:00.0"], visible_bdfs=vis)


def test_cli_validate_resolves_group_through_topology(tmp_path):
    t = _node(4)
    real = "0000:c5:00.0"  # "the" GPU of a 1-GPU box
    t.gpus[3].bdf = real
    path = tmp_path / "topo.json"
    path.write_text(t.to_json())
    out = subprocess.run([sys.executable, "-m", "gpu_topology_on_k8s_amd", "validate", "--resolve-only", "--topology", str(path),
                          "--visible-bdfs", real.upper()], capture_output=True, text=True, cwd=REPO,
                         env={**os.environ, "GTK_GPU_GROUP": "3"}, timeout=120)
    assert out.returncode == 0, out.stderr
    assert json.loads(out.stdout.strip().splitlines()[-1]) == {"hip_devices": [0]}


def test_cli_validate_env_bdfs(capsys):
    rc = cli_main(["validate", "--resolve-only", "--group", "4,5", "--bdfs", "0000:45:00.0,0000:55:00.0",
                   "--visible-bdfs", "0000:55:00.0,0000:45:00.0"])
    assert rc == 0
    assert json.loads(capsys.readouterr().out.strip()) == {"hip_devices": [1, 0]}


def test_visible_view_keeps_measured_matrix_and_masks_hidden():
    t = _node(8)
    bw = np.full((8, 8), 70.0)
    np.fill_diagonal(bw, np.nan)
    bw[6, 7] = bw[7, 6] = 80.0
    t.set_measured_bw(bw, {"method": "p2p_read_lds"})
    vis = [t.gpus[i].bdf for i in (5, 6, 7)]
    view, m, suffix = visible_view(t, 3, vis)
    assert suffix == "" and m.by_bdf
    assert view.n == 8 and np.isfinite(view.bw_gbps[6, 7])  # same node model, same measurements
    assert [g.healthy for g in view.gpus] == [False] * 5 + [True] * 3
    assert all(g.healthy for g in t.gpus)  # the caller's model is untouched


def test_choose_subset_under_visible_devices():
    t = _node(8)
    bw = np.full((8, 8), 70.0)
    np.fill_diagonal(bw, np.nan)
    bw[5, 7] = bw[7, 5] = 90.0  # the best visible pair
    t.set_measured_bw(bw, {"method": "p2p_read_lds"})
    vis = [t.gpus[i].bdf for i in (5, 6, 7)]  # HIP_VISIBLE_DEVICES=5,6,7
    ch = choose_subset(2, topology=t, visible_bdfs=vis)
    assert ch.devices == [5, 7] and ch.hip_devices == [0, 2]
    assert ch.probed and ch.source == "fake" and ch.extra["device_map"]["by_bdf"]
    assert ch.worst is not None and set(ch.worst) <= {5, 6, 7} and ch.worst_hip == [{5: 0, 6: 1, 7: 2}[i] for i in ch.worst]


def test_choose_subset_cpu_visible_count_identity():
    ch = choose_subset(2, visible=4, topology=_node(4))
    assert ch.hip_devices == ch.devices


def test_training_in_a_pod_uses_the_allocated_group(monkeypatch):
    """design.md:239: the workload runs on the devices Allocate handed to the container — rank r on
    GROUP[r], resolved to this container's HIP ordinals by PCI address."""
    from gpu_topology_on_k8s_amd.models.train import _pod_devices

    monkeypatch.setenv("GTK_GPU_GROUP", "6,2")
    monkeypatch.setenv("GTK_GPU_BDFS", "0000:c5:00.0,0000:15:00.0")
    pl = _pod_devices({"rank": 0, "world": 2}, visible_bdfs=["0000:15:00.0", "0000:c5:00.0"])
    assert pl["devices"] == [6, 2] and pl["hip_devices"] == [1, 0] and pl["source"] == "pod-allocation"
    import pytest

    with pytest.raises(ValueError):
        _pod_devices({"rank": 0, "world": 4}, visible_bdfs=["0000:15:00.0", "0000:c5:00.0"])
