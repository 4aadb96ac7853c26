"""Topology model: construction, cost model, (de)serialisation, fixtures F1/F7/F8."""
import json
import math

import numpy as np
import pytest

from gpu_topology_on_k8s_amd.topology import fixtures as fx
from gpu_topology_on_k8s_amd.topology.model import DEFAULT_REF_GBPS, GPUInfo, LinkType, RefLinkClass, Topology, default_link_cost


def test_full_mesh_f7_shape_and_numa():
    t = fx.f7_mi355x()
    assert t.n == 8
    assert (t.link_type[~np.eye(8, dtype=bool)] == int(LinkType.XGMI)).all()
    assert (np.diag(t.hops) == 0).all() and (t.hops[~np.eye(8, dtype=bool)] == 1).all()
    assert t.numa.tolist() == [0, 0, 0, 0, 1, 1, 1, 1]
    # unmeasured xGMI pairs cost one nominal link
    assert np.allclose(t.cost[~np.eye(8, dtype=bool)], 1.0)
    assert all(g.render_minor == 128 + g.index for g in t.gpus)


def test_single_gpu_has_no_pairs():
    """design.md:17-19: with one GPU there is no map[0][0] entry."""
    t = Topology.full_mesh(n=1, numa_split=1)
    assert list(t.pairs()) == []
    assert t.subset_cost([0]) == 0.0


def test_measured_bandwidth_drives_cost():
    t = fx.f7_mi355x(link_gbps=DEFAULT_REF_GBPS)
    assert np.allclose(t.cost[0, 1], 1.0)
    bw = t.bw_gbps.copy()
    bw[2, 5] = DEFAULT_REF_GBPS / 4  # degraded link in one direction only
    t.set_measured_bw(bw, {"method": "test"})
    assert math.isclose(t.cost[2, 5], 4.0) and math.isclose(t.cost[5, 2], 4.0)  # worse direction wins
    assert t.probe["method"] == "test"


def test_cost_falls_back_to_link_class():
    assert default_link_cost(LinkType.SELF) == 0
    assert default_link_cost(LinkType.INTERNAL) < default_link_cost(LinkType.XGMI) < default_link_cost(LinkType.PCIE)
    assert default_link_cost(LinkType.PCIE) < default_link_cost(LinkType.PCIE_SYS) < default_link_cost(LinkType.UNKNOWN)
    assert default_link_cost(LinkType.XGMI, hops=2) == 2.0


def test_json_roundtrip_preserves_everything():
    t = fx.f7_mi355x(link_gbps=70.0, noise=0.1, seed=3)
    t.hbm_gbps = np.array([3000.0] * 7 + [np.nan])
    t.probe = {"method": "p2p_read_lds", "ts": 1}
    u = Topology.from_json(t.to_json())
    assert np.allclose(u.cost, t.cost)
    assert np.allclose(u.bw_gbps, t.bw_gbps, equal_nan=True)
    assert np.isnan(u.hbm_gbps[7]) and u.hbm_gbps[0] == 3000.0
    assert [g.numa for g in u.gpus] == [g.numa for g in t.gpus]
    assert u.probe == t.probe
    json.loads(t.to_json())  # strict JSON (no NaN literals)
    assert "NaN" not in t.to_json()


def test_validation_rejects_bad_matrices():
    gpus = [GPUInfo(index=0), GPUInfo(index=1)]
    with pytest.raises(ValueError):
        Topology(gpus=gpus, link_type=[[0, 2], [3, 0]], hops=[[0, 1], [1, 0]])
    with pytest.raises(ValueError):
        Topology(gpus=[GPUInfo(index=0), GPUInfo(index=2)], link_type=[[0, 2], [2, 0]], hops=[[0, 1], [1, 0]])
    with pytest.raises(ValueError):
        Topology(gpus=gpus, link_type=[[0, 2], [2, 0]], hops=[[0, 1], [1, 0]], cost=[[0, -1], [-1, 0]])


def test_f1_reference_matrix():
    t = fx.f1_nvlink_host()
    assert RefLinkClass(int(t.ref_class[0, 1])) == RefLinkClass.NV3
    assert RefLinkClass(int(t.ref_class[0, 2])) == RefLinkClass.PHB
    # NV3 ring: every GPU has exactly two NV3 neighbours
    nv = (t.ref_class == int(RefLinkClass.NV3)).sum(axis=1)
    assert nv.tolist() == [2] * 8
    assert t.cost[0, 1] < t.cost[0, 2]
    assert all(g.cpu_affinity == "0-63" for g in t.gpus)


def test_f8_cpx_partitions():
    t = fx.f8_mi355x_cpx()
    assert t.n == 64
    assert t.physical.tolist() == [i // 8 for i in range(64)]
    assert LinkType(int(t.link_type[0, 1])) == LinkType.INTERNAL
    assert LinkType(int(t.link_type[0, 8])) == LinkType.XGMI
    assert t.cost[0, 1] < t.cost[0, 8]
    assert all(g.partition == "CPX" for g in t.gpus)


def test_render_table():
    t = fx.f7_mi355x(link_gbps=76.0)
    s = t.render()
    assert s.splitlines()[0].strip().startswith("GPU0")
    assert "XGMI" in s and len(s.splitlines()) == 9
