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
    assert out["config"]["parallelism"] == "dp2"


def test_bench_single_rank_cpu():
    out = _bench("--backend", "cpu", "--steps", "2", "--warmup", "1", "--size-mb", "1")
    assert out["n_gpus"] == 1 and out["busbw_gbps"] == 0.0 and out["value"] == out["algbw_gbps"]


def test_parse_ctas():
    sys.path.insert(0, REPO)
    import bench

    assert bench.parse_ctas("auto") is None and bench.parse_ctas("default") is None
    assert bench.parse_ctas("64") == (64, 0) and bench.parse_ctas("32:64") == (32, 64)
    assert (0, 0) in bench.TUNE_CANDIDATES
