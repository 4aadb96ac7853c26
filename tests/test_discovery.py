"""Native discovery (``_topo``) against synthetic KFD sysfs trees, and the discovery front-end."""
import numpy as np
import pytest

from gpu_topology_on_k8s_amd._native import available, load
from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.discovery import DiscoveryError, discover, fake_topology, from_native
from gpu_topology_on_k8s_amd.topology.model import LinkType, Topology

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


# ------------------------------------------------------------------ amdsmi backend on a stand-in library
def _fake_amdsmi():
    from gpu_topology_on_k8s_amd._native import binary

    try:
        return str(binary("libfake_amdsmi.so"))
    except Exception:
        pytest.skip("fake_amdsmi not built")


def _amdsmi_node(monkeypatch, tmp_path, **env):
    for k in ("FAKE_AMDSMI_GPUS", "FAKE_AMDSMI_PARTITIONS", "FAKE_AMDSMI_HIP_ORDER", "FAKE_AMDSMI_DOWN"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(f"FAKE_AMDSMI_{k.upper()}", str(v))
    return discover("amdsmi", amdsmi_lib=_fake_amdsmi(), pci_root=str(tmp_path), node_root=str(tmp_path))


@needs_topo
def test_amdsmi_backend_eight_gpu_mesh(monkeypatch, tmp_path):
    """The pairwise half of the amdsmi reader (what bench.py's rank 0 runs on the 8-GPU node)."""
    t = _amdsmi_node(monkeypatch, tmp_path)
    off = ~np.eye(8, dtype=bool)
    assert t.n == 8 and t.source == "amdsmi"
    assert (t.link_type[off] == int(LinkType.XGMI)).all() and (t.hops[off] == 1).all()
    assert (t.weight[off] == 15).all() and t.probe["amdsmi_max_bw_mbps"][0][1] == 76800
    assert t.numa.tolist() == [0] * 4 + [1] * 4 and all(g.xgmi_links_up == 7 for g in t.gpus)
    assert all(g.gfx == "gfx950" and g.model == "MI355X" and g.render_minor == 128 + i for i, g in enumerate(t.gpus))
    assert len({g.bdf for g in t.gpus}) == 8


@needs_topo
def test_amdsmi_backend_orders_by_hip_id_and_maps_bdfs(monkeypatch, tmp_path):
    t = _amdsmi_node(monkeypatch, tmp_path, hip_order="3,2,1,0,4,5,6,7")
    assert [g.bdf for g in t.gpus][:4] == ["0000:35:00.0", "0000:25:00.0", "0000:15:00.0", "0000:05:00.0"]
    from gpu_topology_on_k8s_amd.parallel.allreduce import choose_subset

    ch = choose_subset(2, topology=t, visible_bdfs=["0000:45:00.0", "0000:55:00.0"])  # HIP_VISIBLE_DEVICES=4,5
    assert ch.devices == [4, 5] and ch.hip_devices == [0, 1]


@needs_topo
def test_amdsmi_backend_down_link(monkeypatch, tmp_path):
    t = _amdsmi_node(monkeypatch, tmp_path, down="2-6")
    assert LinkType(int(t.link_type[2, 6])) == LinkType.PCIE_SYS and t.hops[2, 6] == 2
    assert t.gpus[2].xgmi_links_up == 6 and t.gpus[6].xgmi_links_up == 6 and t.gpus[0].xgmi_links_up == 7
    assert t.cost[2, 6] > t.cost[2, 5]
    from gpu_topology_on_k8s_amd.placement import select

    assert set(select(t, 2, used=[0, 1, 3, 4, 5]).ids) in ({2, 7}, {6, 7})  # the down pair is avoided


@needs_topo
def test_amdsmi_backend_cpx(monkeypatch, tmp_path):
    t = _amdsmi_node(monkeypatch, tmp_path, partitions=8)
    assert t.n == 64 and t.physical.tolist() == [i // 8 for i in range(64)]
    assert all(g.partition == "CPX" for g in t.gpus)
    assert LinkType(int(t.link_type[0, 1])) == LinkType.INTERNAL and LinkType(int(t.link_type[0, 8])) == LinkType.XGMI
    from gpu_topology_on_k8s_amd.k8s.annotations import annotations_size, encode_node_annotations

    ann = encode_node_annotations(t)
    assert annotations_size(ann) < 64 * 1024 and sum(k.startswith("GPUPKG_") for k in ann) == 28


def test_probe_pairs_per_package_on_cpx():
    """A CPX node is probed per package pair (72 copies instead of 4096) and every XCP pair takes its
    packages' number, so the XCPs of a package stay interchangeable for the placement engine."""
    from gpu_topology_on_k8s_amd.ops.probe import _probe_pairs
    from gpu_topology_on_k8s_amd.topology import fixtures as fx

    t = fx.f8_mi355x_cpx()
    pairs, rep = _probe_pairs(t, list(range(64)), by_package=True)
    assert len(pairs) == 8 + 8 + 56 and len(set(pairs)) == len(pairs)
    phys = t.physical
    for (i, j), (a, b) in rep.items():
        assert (a, b) in pairs
        assert phys[a] == phys[i] and phys[b] == phys[j]
        assert (i == j) == (a == b)
    full, none = _probe_pairs(t, list(range(64)), by_package=False)
    assert none is None and len(full) == 64 * 64
    flat, r8 = _probe_pairs(fx.f7_mi355x(), list(range(8)), by_package=True)  # unpartitioned: every pair
    assert r8 is None and len(flat) == 64


@needs_topo
def test_sysfs_nics_pcie_classes_and_nearest(tmp_path):
    """RDMA NICs from /sys/class/infiniband and the reference's PCIe taxonomy per GPU-NIC pair: the NIC on
    the GPU's own switch is PIX, the same socket's others PHB, the other socket's SYS."""
    p = fx.write_fake_kfd_sysfs(str(tmp_path), nics=True)
    t = from_native(load("_topo").discover_sysfs(p["kfd"], p["drm"], p["pci"], p["node"], p["ib"]))
    assert [n["name"] for n in t.nics] == [f"ionic_{i}" for i in range(8)]
    assert t.nics[0]["rate_gbps"] == 400.0 and "ACTIVE" in t.nics[0]["state"] and t.nics[0]["netdev"]
    assert t.gpu_nic[0][0] == 1 and t.gpu_nic[0][1] == 3 and t.gpu_nic[0][4] == 5
    assert t.nearest_nics([1, 6]) == ["ionic_1", "ionic_6"]
    # survives the node annotation codec
    back = Topology.from_json(t.to_wire())
    assert back.nearest_nics([3]) == ["ionic_3"] and back.gpu_nic == t.gpu_nic
    # a down port loses to an active one of the same class
    t.nics[2]["state"] = "1: DOWN"
    t.gpu_nic[2][3] = 1
    assert t.nearest_nics([2]) == ["ionic_3"]
    # no NIC tree: nothing
    q = fx.write_fake_kfd_sysfs(str(tmp_path / "plain"))
    t2 = from_native(load("_topo").discover_sysfs(q["kfd"], q["drm"], q["pci"], q["node"], str(tmp_path / "none")))
    assert not t2.nics and t2.nearest_nics([0]) == []
