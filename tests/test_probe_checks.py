"""The self-validation the first 8-GPU run relies on (ops/checks.py): fed a node
whose every link runs at PCIe rate (peer access fallen back to host staging on all pairs alike) and a
gather that serialises its sources, both are flagged, although each looks fine against its siblings."""
import numpy as np

from gpu_topology_on_k8s_amd.ops.checks import check_gather, check_pairs, check_ring, matrix_rates, rated_link_gbps
from gpu_topology_on_k8s_amd.topology import fixtures as fx


def _node(rate, amdsmi_mbps=153_600):
    t = fx.f7_mi355x()
    bw = np.full((t.n, t.n), float(rate))
    np.fill_diagonal(bw, np.nan)
    t.probe["amdsmi_max_bw_mbps"] = [[0 if i == j else amdsmi_mbps for j in range(t.n)] for i in range(t.n)]
    t.set_measured_bw(bw, {"method": "p2p_read_lds"})
    return t


def test_healthy_xgmi_node_passes():
    t = _node(64.0)
    assert rated_link_gbps(t, 0, 1) == 76.8  # amdsmi's bidirectional figure, per direction (kept across the probe)
    assert check_pairs(t, matrix_rates(t)) == []
    assert check_gather(7 * 60.0, [64.0] * 7) == []
    assert check_ring(0.9 * 7 * 64.0, 7 * 64.0) == []


def test_every_link_at_pcie_rate_is_flagged():
    """Uniformly slow links pass a median-relative floor; the amdsmi-rated one catches them."""
    t = _node(25.0)
    probs = check_pairs(t, matrix_rates(t))
    assert len(probs) == t.n * (t.n - 1) and "below its floor 38.4" in probs[0]


def test_one_degraded_link_is_flagged_and_nominal_rate_applies_without_amdsmi():
    t = _node(64.0)
    t.probe.pop("amdsmi_max_bw_mbps")
    assert rated_link_gbps(t, 0, 1) == 76.8  # the xGMI class's nominal rate
    bw = t.bw_gbps.copy()
    bw[2, 5] = 20.0
    t.set_measured_bw(bw, {"method": "p2p_read_lds"})
    probs = check_pairs(t, matrix_rates(t))
    assert len(probs) == 1 and probs[0].startswith("pair 2->5")


def test_serialised_gather_and_weak_ring_are_flagged():
    single = [62.0, 64.0, 63.0, 65.0, 61.0, 64.0, 60.0]
    assert check_gather(70.0, single)  # one link's worth from 7 sources: serialised
    assert check_gather(0.9 * 63.0 * 3, single)  # still under half of 7 links
    assert check_ring(0.3 * 448.0, 448.0)  # what the old 0.3 floor let through
    assert check_ring(1.3 * 448.0, 448.0)  # above the bound: the pair reads are wrong
