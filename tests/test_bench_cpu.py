"""bench.py driver contract on CPU: the N>1 path (torch.distributed.run relaunch, rank-0 placement via
the store, barrier-bracketed timing, max over ranks, one JSON line) exercised with gloo."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True, timeout=timeout,
                       cwd=REPO, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_bench_two_ranks_gloo():
    out = _bench("--gpus", "2", "--backend", "cpu", "--steps", "3", "--warmup", "1", "--size-mb", "1")
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config"):
        assert key in out
    assert out["metric"] == "RCCL all-reduce bus GB/s on scheduler-chosen k-GPU subset, k=1/2/4/8"
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["higher_is_better"] is True and out["scaling"] == "weak"
    assert len(set(out["config"]["subset"])) == 2
    assert out["value"] > 0 and abs(out["busbw_gbps"] - out["algbw_gbps"]) < 1e-3 * out["algbw_gbps"] + 1e-6  # 2(k-1)/k = 1
    assert abs(out["value"] - 2 * out["busbw_gbps"]) <= 1e-2 * out["value"] + 2e-3  # whole-job aggregate of 2 ranks
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["message_bytes_per_gpu"] == 1 << 20
    k8s = out["k8s_placement"]  # placed through device plugin + extender + kubelet Allocate
    assert k8s["devices"] == out["config"]["subset"] and k8s["assigned"] is True
    assert k8s["group_annotation"] == ",".join(str(i) for i in out["config"]["subset"])
    sw = out["size_sweep"]
    assert sw["all_exact"] and [r["bytes"] for r in sw["rows"]][:2] == [8, 64] and sw["peak"]["busbw_gbps"] > 0


def test_bench_line_is_internally_consistent():
    """The numbers of the JSON line agree with each other and with the timed phase: algBW is the message
    over ms_per_step, busBW is algBW x 2(k-1)/k, the value is k x busBW, and ms_per_step x steps of the
    timed region fits inside the headline phase (the driver checks the line against its own clock)."""
    steps = 40
    out = _bench("--gpus", "2", "--backend", "cpu", "--steps", str(steps), "--warmup", "1", "--size-mb", "4",
                 "--sweep", "off", "--probe", "off")
    k, nbytes, ms = out["n_gpus"], out["config"]["message_bytes_per_gpu"], out["ms_per_step"]
    algbw = nbytes / (ms / 1e3) / 1e9
    rel = 1e-4 / ms + 1e-6  # ms_per_step is printed to 4 decimals
    assert abs(out["algbw_gbps"] - algbw) <= rel * algbw + 2e-3, out
    assert abs(out["busbw_gbps"] - algbw * 2 * (k - 1) / k) <= rel * algbw + 2e-3, out
    assert abs(out["value"] - k * out["busbw_gbps"]) <= 2e-2 * out["value"] + 4e-3, out
    # the headline phase is the timed region plus its bracketing barriers, on rank 0's clock (rounded to ms)
    assert ms * steps <= out["phase_s"]["headline"] * 1e3 + 0.5, out


def test_bench_single_rank_cpu():
    out = _bench("--backend", "cpu", "--steps", "2", "--warmup", "1", "--size-mb", "1", "--via", "direct")
    assert out["k8s_placement"] is None
    assert out["n_gpus"] == 1 and out["busbw_gbps"] == 0.0 and out["value"] == out["algbw_gbps"]
    # the k=1 point says it is a copy rate, not comparable to k>=2 aggregate busBW
    assert out["scaling_comparable"] is False and "not comparable" in out["scaling_note"]
    assert out["aggregate_busbw_gbps"] is None and out["per_rank_busbw_gbps"] is None


def test_parse_ctas():
    sys.path.insert(0, REPO)
    import bench

    assert bench.parse_ctas("auto") is None and bench.parse_ctas("default") is None
    assert bench.parse_ctas("64") == (64, 0) and bench.parse_ctas("32:64") == (32, 64)
    assert (0, 0) in bench.TUNE_CANDIDATES


def test_choose_subset_uses_probed_topology():
    """A probed node (measured GB/s) steers the k=2 choice to the fastest pair and is summarised."""
    import numpy as np

    sys.path.insert(0, REPO)
    from gpu_topology_on_k8s_amd.parallel.allreduce import choose_subset, probe_summary
    from gpu_topology_on_k8s_amd.topology.discovery import fake_topology

    topo = fake_topology(4)
    bw = np.full((4, 4), 50.0)
    bw[2, 3] = bw[3, 2] = 70.0  # one faster link
    np.fill_diagonal(bw, np.nan)
    topo.set_measured_bw(bw, {"method": "p2p_read_lds", "preset": "quick"})
    ch = choose_subset(2, visible=4, topology=topo)
    assert sorted(ch.devices) == [2, 3] and ch.probed
    s = ch.extra["probe"]
    assert s["link_read_gbps"]["pairs"] == 12 and s["link_read_gbps"]["max"] == 70.0
    assert s["subset_link_read_gbps"] == {"min": 70.0, "max": 70.0}
    assert probe_summary(topo, [0, 1])["subset_link_read_gbps"]["max"] == 50.0


def test_probe_node_failure_is_reported_not_raised():
    sys.path.insert(0, REPO)
    from gpu_topology_on_k8s_amd.parallel.allreduce import probe_node

    topo, msg = probe_node("quick", backend="fake", timeout=120)
    assert topo is None and "probe" in msg


def test_sweep_sizes():
    sys.path.insert(0, REPO)
    import bench

    assert bench.sweep_sizes("off") == []
    full = bench.sweep_sizes("auto")
    assert full[0] == 8 and full[-1] == 16 << 30 and full[-2] == 8 << 30
    assert bench.sweep_sizes("auto", cpu=True)[-1] == 1 << 20
    assert bench.sweep_sizes("1K:4K:2") == [1024, 2048, 4096]


def test_ingress_bound():
    import numpy as np

    sys.path.insert(0, REPO)
    from gpu_topology_on_k8s_amd.ops.probe import ingress_bound
    from gpu_topology_on_k8s_amd.topology.discovery import fake_topology

    topo = fake_topology(4)
    assert ingress_bound(topo, [0, 1]) is None  # nothing measured
    bw = np.full((4, 4), 60.0)
    np.fill_diagonal(bw, np.nan)
    topo.set_measured_bw(bw, {"method": "p2p_read_lds"})
    assert ingress_bound(topo, [0]) is None
    assert ingress_bound(topo, [0, 1]) == 60.0
    assert ingress_bound(topo, [0, 1, 2, 3]) == 180.0  # 3 links per member
    topo.probe["ingress_all_gbps"] = [150.0, 170.0, None, 175.0]  # shared fabric caps member 0
    assert ingress_bound(topo, [0, 1, 2, 3]) == 150.0


def test_bench_eight_ranks_gloo_dry_run():
    """The N=8 driver run, rehearsed on CPU: 8 ranks, an 8-device fake node placed through the full
    k8s flow (k = n: no worst subset), the store protocol with 8 ranks, max-over-ranks timing."""
    out = _bench("--gpus", "8", "--backend", "cpu", "--discovery", "fake", "--steps", "2", "--warmup", "1", "--size-mb", "1",
                 "--sweep", "8:64K:64", timeout=900)
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert sorted(out["config"]["subset"]) == list(range(8)) and out["config"]["worst_subset"] is None
    assert out["k8s_placement"]["assigned"] is True and len(out["k8s_placement"]["devices"]) == 8
    assert abs(out["busbw_gbps"] - out["algbw_gbps"] * 2 * 7 / 8) <= 1e-2 * out["busbw_gbps"] + 2e-3  # 3-decimal rounding
    assert out["size_sweep"]["all_exact"] and out["value_kind"].startswith("aggregate busbw")
    assert abs(out["value"] - 8 * out["busbw_gbps"]) <= 1e-2 * out["value"] + 2e-2  # every rank's busBW summed
    assert out["scaling_comparable"] is True and out["aggregate_busbw_gbps"] == out["value"]
    assert out["per_rank_busbw_gbps"] == out["busbw_gbps"]
    ph = out["phase_s"]  # the first 8-GPU run explains itself: where its wall time went
    for key in ("place", "comm", "check", "warmup", "headline", "sweep", "total"):
        assert key in ph and ph[key] >= 0, ph
    assert ph["total"] >= ph["headline"] and out["skipped_phases"] == []
    assert len(out["cpuset_applied"]) == 8 and all("applied" in b for b in out["cpuset_applied"])


def test_bench_tiny_budget_keeps_the_headline():
    """--budget-s far below any phase's cost: every supplementary phase is skipped by all ranks
    together, and the headline line still comes out, measured."""
    out = _bench("--gpus", "2", "--backend", "cpu", "--steps", "2", "--warmup", "1", "--size-mb", "1", "--budget-s", "0.001")
    assert out["value"] > 0 and out["steps"] == 2 and out["phase_s"]["headline"] > 0
    skipped = {s["phase"] for s in out["skipped_phases"]}
    assert "sweep" in skipped and out["size_sweep"] is None
    assert "ab_worst" not in out["phase_s"] and "sweep" not in out["phase_s"]


def test_bench_four_ranks_on_amdsmi_discovered_node():
    """N=4 of an 8-GPU node discovered through the amdsmi reader (stand-in library): placement picks a
    4-subset of the 8 real-shaped devices, with a worst subset, through the k8s flow."""
    from gpu_topology_on_k8s_amd._native import binary

    lib = str(binary("libfake_amdsmi.so"))
    env = dict(os.environ, GTK_AMDSMI_LIB=lib)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--backend", "cpu", "--discovery", "amdsmi",
                        "--steps", "2", "--warmup", "1", "--size-mb", "1", "--sweep", "off", "--cpu-visible", "8"],
                       capture_output=True, text=True, timeout=600, cwd=REPO, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    cfg = out["config"]
    assert cfg["topology_source"].startswith("amdsmi") and len(cfg["subset"]) == 4
    assert cfg["worst_subset"] is not None and cfg["worst_score"] < cfg["placement_score"]
    assert out["k8s_placement"]["assigned"] is True
    # the placement A/B of the same run: a second communicator timed on the worst 4-subset
    ab = out["worst_subset_ab"]
    assert ab and "error" not in ab, ab
    assert ab["subset"] == cfg["worst_subset"] and ab["exact"] and ab["busbw_gbps"] > 0
    assert out["placement_gain"] is not None and out["placement_gain"] > 0


def test_rccl_log_summary_parses_transports():
    """bench.py reports how RCCL carried every ring edge (k >= 2) from its INFO log."""
    from gpu_topology_on_k8s_amd.parallel.allreduce import rccl_log_env, rccl_log_summary

    env = rccl_log_env("/tmp/x")
    assert env["NCCL_DEBUG"] == "INFO" and env["NCCL_DEBUG_FILE"].endswith(".%p")
    text = "\n".join([
        "node:123:123 [0] NCCL INFO RCCL version 2.27.7-HEAD:abc",
        "node:123:130 [0] NCCL INFO comm 0x5555 rank 0 nRanks 2 nNodes 1 localRanks 2 localRank 0 MNNVL 0",
        "node:123:130 [0] NCCL INFO Channel 00/32 : 0[0] -> 1[1] via P2P/IPC",
        "node:123:130 [0] NCCL INFO Channel 01/32 : 0[0] -> 1[1] via P2P/IPC",
        "node:123:130 [0] NCCL INFO Channel 00/0 : 0[2a000] -> 1[3a000] via P2P/direct pointer comm 0x5555",
        "node:123:130 [0] NCCL INFO 32 coll channels, 32 collnet channels, 0 nvls channels, 32 p2p channels, 2 p2p channels per peer",
    ])
    s = rccl_log_summary(text)
    assert s["communicators"] == 1 and s["nranks"] == [2] and s["coll_channels"] == [32]
    assert s["edges_via"]["P2P/IPC"] == 2 and "RCCL version 2.27.7" in s["version"]
    assert s["p2p_only"] is True and s["non_p2p_edges"] == {}


def test_rccl_log_summary_flags_a_broken_transport():
    """What an NCCL_P2P_DISABLE=1 run logs: ring edges through host shared memory.  The summary says
    the ring left xGMI peer access, which the k >= 2 GPU test asserts against."""
    from gpu_topology_on_k8s_amd.parallel.allreduce import rccl_log_summary

    text = "\n".join([
        "node:9:9 [0] NCCL INFO comm 0x77 rank 0 nRanks 2 nNodes 1 localRanks 2 localRank 0 MNNVL 0",
        "node:9:9 [0] NCCL INFO Channel 00/02 : 0[0] -> 1[1] via SHM/direct/direct",
        "node:9:9 [0] NCCL INFO Channel 01/02 : 0[0] -> 1[1] via SHM/direct/direct",
        "node:9:9 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC",
    ])
    s = rccl_log_summary(text)
    assert s["p2p_only"] is False and s["non_p2p_edges"] == {"SHM/direct/direct": 2}
    assert rccl_log_summary("")["p2p_only"] is False  # no edges logged proves nothing


def test_watchdog_reports_the_stuck_phase_and_exits():
    """A hung collective cannot be interrupted from Python: the watchdog prints rank 0's JSON line with
    value null and the phase in progress, dumps the thread stacks and exits 124 (here into buffers,
    with the exit captured)."""
    import io
    import threading
    import time as _time

    sys.path.insert(0, REPO)
    import bench

    args = bench.parse(["--steps", "3", "--warmup", "1"])
    ph = bench.Phases(300.0)
    out, err, codes = io.StringIO(), io.StringIO(), []
    done = threading.Event()

    def fake_exit(code):
        codes.append(code)
        done.set()

    stuck = threading.Thread(target=lambda: ph.run("headline", done.wait, 30), daemon=True)
    stuck.start()
    _time.sleep(0.05)
    t = bench.start_watchdog(0.2, ph, 0, 8, args, exit_fn=fake_exit, out=out, err=err)
    assert done.wait(10) and codes == [124]
    line = json.loads(out.getvalue().strip().splitlines()[-1])
    assert line["value"] is None and line["n_gpus"] == 8 and "'headline'" in line["error"]
    assert line["metric"] == "RCCL all-reduce bus GB/s on scheduler-chosen k-GPU subset, k=1/2/4/8"
    assert "thread stacks follow" in err.getvalue()
    t.cancel()
    assert bench.start_watchdog(0, ph, 0, 1, args) is None


def test_watchdog_after_the_headline_keeps_the_measured_value():
    """A supplementary phase (size sweep, fp32, graph latency, worst-subset A/B) that hangs after the
    headline was timed must not cost the measurement: the watchdog's line carries the headline value and
    contract fields, with the stuck phase named in ``error``."""
    import io
    import threading
    import time as _time

    sys.path.insert(0, REPO)
    import bench

    args = bench.parse(["--steps", "3", "--warmup", "1"])
    ph = bench.Phases(300.0)
    ph.headline = {"metric": bench.METRIC, "value": 1234.5, "unit": "GB/s", "n_gpus": 2, "steps": 3, "warmup": 1,
                   "ms_per_step": 1.7, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
                   "config": {"model": "rccl-allreduce", "parallelism": "dp2"}}
    out, err, codes = io.StringIO(), io.StringIO(), []
    done = threading.Event()

    def fake_exit(code):
        codes.append(code)
        done.set()

    stuck = threading.Thread(target=lambda: ph.run("ab_worst", done.wait, 30), daemon=True)
    stuck.start()
    _time.sleep(0.05)
    t = bench.start_watchdog(0.2, ph, 0, 2, args, exit_fn=fake_exit, out=out, err=err)
    assert done.wait(10) and codes == [124]
    line = json.loads(out.getvalue().strip().splitlines()[-1])
    assert line["value"] == 1234.5 and line["ms_per_step"] == 1.7 and line["config"]["parallelism"] == "dp2"
    assert "'ab_worst'" in line["error"] and "after the headline" in line["error"]
    t.cancel()
