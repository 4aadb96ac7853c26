"""Native discovery (``_topo``) against synthetic KFD sysfs trees, and the discovery front-end."""
import numpy as np
import pytest

from gpu_topology_on_k8s_amd._native import available, load
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.discovery import DiscoveryError, discover, fake_topology, from_native
from gpu_topology_on_k8s_amd.topology.model import LinkType

needs_topo = pytest.mark.skipif(not available("_topo"), reason="_topo not built")


@needs_topo
def test_sysfs_full_mesh(tmp_path):
    p = fx.write_fake_kfd_sysfs(str(tmp_path))
    d = load("_topo").discover_sysfs(p["kfd"], p["drm"], p["pci"], p["node"])
    assert d["source"] == "sysfs"
    assert len(d["gpus"]) == 8
    g0 = d["gpus"][0]
    assert g0["gfx"] == "gfx950" and g0["model"] == "MI355X"
    assert g0["render_minor"] == 128 and g0["card"] == 0
    assert g0["xgmi_links_up"] == 7 and g0["cus"] == 256
    t = from_native(d, node_name="n1")
    assert (t.link_type[~np.eye(8, dtype=bool)] == int(LinkType.XGMI)).all()
    assert (t.hops[~np.eye(8, dtype=bool)] == 1).all()
    assert t.numa.tolist() == [0, 0, 0, 0, 1, 1, 1, 1]
    assert not d["warnings"]


@needs_topo
def test_sysfs_ras_counters(tmp_path):
    """amdgpu ras/<block>_err_count files are summed per device; retired pages counted; absent = -1."""
    p = fx.write_fake_kfd_sysfs(str(tmp_path), ras={1: {"umc": (2, 5), "gfx": (1, 0), "bad_pages": 3}})
    t = from_native(load("_topo").discover_sysfs(p["kfd"], p["drm"], p["pci"], p["node"]))
    g1, g0 = t.gpus[1], t.gpus[0]
    assert (g1.ecc_uncorrectable, g1.ecc_correctable, g1.bad_pages) == (3, 5, 3)
    assert (g0.ecc_uncorrectable, g0.ecc_correctable, g0.bad_pages) == (-1, -1, -1)
    assert g0.xgmi_links_total == g0.xgmi_links_up == 7


@needs_topo
def test_sysfs_missing_xgmi_link_falls_back_to_pcie(tmp_path):
    p = fx.write_fake_kfd_sysfs(str(tmp_path), missing_links=[(0, 5)])
    t = from_native(load("_topo").discover_sysfs(p["kfd"], p["drm"], p["pci"], p["node"]))
    assert LinkType(int(t.link_type[0, 5])) == LinkType.PCIE_SYS
    assert t.cost[0, 5] > t.cost[0, 1]
    assert t.gpus[0].xgmi_links_up == 6


@needs_topo
def test_sysfs_cpx_partitions(tmp_path):
    p = fx.write_fake_kfd_sysfs(str(tmp_path), partitions_per_gpu=8)
    t = from_native(load("_topo").discover_sysfs(p["kfd"], p["drm"], p["pci"], p["node"]))
    assert t.n == 64
    assert t.physical.tolist() == [i // 8 for i in range(64)]
    assert all(g.partition == "CPX" for g in t.gpus)
    assert LinkType(int(t.link_type[0, 1])) == LinkType.INTERNAL
    assert LinkType(int(t.link_type[0, 8])) == LinkType.XGMI


@needs_topo
def test_sysfs_empty_root_raises(tmp_path):
    with pytest.raises(RuntimeError):
        load("_topo").discover_sysfs(str(tmp_path), str(tmp_path))


@needs_topo
def test_amdsmi_missing_library_raises():
    with pytest.raises(RuntimeError):
        load("_topo").discover_amdsmi("libdefinitely_not_amdsmi.so")


def test_discover_fake_backend():
    t = discover("fake", fake_n=2)
    assert t.n == 2 and t.source == "fake"
    assert fake_topology(8).numa.tolist() == [0] * 4 + [1] * 4


@needs_topo
def test_discover_sysfs_via_frontend(tmp_path):
    p = fx.write_fake_kfd_sysfs(str(tmp_path), n_gpus=4, sockets=1)
    t = discover("sysfs", sysfs_root=p["kfd"], drm_root=p["drm"], node_name="x", pci_root=p["pci"], node_root=p["node"])
    assert t.n == 4 and t.node_name == "x"


def test_discover_never_silently_fakes(tmp_path):
    with pytest.raises(DiscoveryError):
        discover("sysfs", sysfs_root=str(tmp_path / "nope"), drm_root=str(tmp_path))


@needs_topo
def test_sysfs_host_affinity(tmp_path):
    """local_cpulist, PCIe link training and NUMA SLIT distances (CPU-affinity inputs, design.md:144-145)."""
    p = fx.write_fake_kfd_sysfs(str(tmp_path), degraded_pcie=[2])
    t = from_native(load("_topo").discover_sysfs(p["kfd"], p["drm"], p["pci"], p["node"]))
    assert t.gpus[0].cpu_affinity == "0-47,96-143" and t.gpus[7].cpu_affinity == "48-95,144-191"
    assert t.gpus[2].pcie_link_ratio == 0.5 and t.gpus[3].pcie_link_ratio == 1.0
    assert t.numa_distance == {0: [10, 32], 1: [32, 10]}
    c = fx.write_fake_kfd_sysfs(str(tmp_path / "cpx"), partitions_per_gpu=8)
    tc = from_native(load("_topo").discover_sysfs(c["kfd"], c["drm"], c["pci"], c["node"]))
    assert tc.gpus[9].cpu_affinity == "0-47,96-143"  # XCP function 1: read through function 0
