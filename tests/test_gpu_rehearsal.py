"""GPU, one MI355X: the multi-rank data-parallel GPU code paths rehearsed with two ranks on the one
GPU (``GTK_REHEARSE_ON_ONE_GPU=1``: collectives over gloo, since RCCL refuses two ranks on one
device).  Bucketed gradient all-reduce from backward hooks, ZeRO-1's reduce-scatter + sharded HIP
AdamW + per-bucket weight all-gather, and MNIST DP all run with world size 2 on real HIP kernels,
and must reproduce the one-rank losses (same data on both ranks).  The RCCL versions of these runs
are tests/test_gpu_multi.py (>= 2 GPUs)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, port=None, timeout=600):
    e = dict(os.environ, GTK_REHEARSE_ON_ONE_GPU="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    cmd = [sys.executable]
    if port:
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1", f"--master-port={port}"]
    cmd += ["-m", "gpu_topology_on_k8s_amd.models.train", *args]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO, env=e)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("zero1", [False, True])
def test_two_ranks_on_one_gpu_match_one_rank_llama(zero1):
    base = ["--model", "tiny", "--batch", "2", "--seq", "128", "--steps", "3", "--warmup", "1", "--same-data",
            "--gemm-tuning", "off", "--bucket-mb", "1"] + (["--zero1"] if zero1 else [])
    one = _run(base)
    two = _run(base, port=29631 + int(zero1))
    assert two["n_gpus"] == 2 and two["placement_source"] == "rehearsal" and len(two["losses"]) == len(one["losses"])
    for a, b in zip(one["losses"], two["losses"]):
        assert abs(a - b) <= 2e-2 * max(1.0, abs(a)), (one["losses"], two["losses"])
    print(json.dumps({"zero1": zero1, "one_rank": one["losses"], "two_ranks": two["losses"]}))


def test_two_ranks_on_one_gpu_match_one_rank_mnist():
    base = ["--model", "mnist-cnn", "--batch", "64", "--steps", "5", "--warmup", "1", "--same-data", "--graph", "off",
            "--gemm-tuning", "off"]
    one = _run(base)
    two = _run(base, port=29635)
    for a, b in zip(one["losses"], two["losses"]):
        assert abs(a - b) <= 2e-2 * max(1.0, abs(a)), (one["losses"], two["losses"])
    print(json.dumps({"one_rank": one["losses"], "two_ranks": two["losses"]}))
