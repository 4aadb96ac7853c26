"""GPU, one MI355X: the multi-rank data-parallel GPU code paths rehearsed with two ranks on the one
GPU (``GTK_REHEARSE_ON_ONE_GPU=1``: collectives over gloo, since RCCL refuses two ranks on one
device).  Bucketed gradient all-reduce from backward hooks, ZeRO-1's reduce-scatter + sharded update
+ per-bucket weight all-gather, the fp32 reduction and MNIST DP all run with world size 2 on real HIP
kernels, with DIFFERENT data per rank: the first reduction is checked against the exact sum of both
ranks' local gradients and the SGD weight update against a 1-rank job on the concatenated batch.  The
RCCL versions of these runs are tests/test_gpu_multi.py (>= 2 GPUs)."""
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
    tb = p.stderr.find("Traceback")  # the first rank's traceback, not the launcher's summary
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[tb:tb + 4000] if tb >= 0 else p.stderr[-4000:])
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def _rel(a, b):
    import math

    d = math.sqrt(sum((x - y) ** 2 for x, y in zip(a, b)))
    return d / max(1e-30, math.sqrt(sum(y * y for y in b)))


COMMON = ["--steps", "2", "--warmup", "1", "--gemm-tuning", "off", "--optimizer", "sgd", "--lr", "0.5", "--fingerprint"]


@pytest.mark.parametrize("case", ["llama", "llama-zero1", "llama-fp32", "mnist"])
def test_two_ranks_on_one_gpu_reduce_exactly_and_match_the_concatenated_batch(case):
    """Different data per rank: the 2-rank job's first reduction against the fp64
    sum of both ranks' local gradients (--check-reduction), and its SGD weight-update fingerprint
    against a 1-rank job on the concatenated batch (--data-ranks 2)."""
    args = {"llama": ["--model", "tiny", "--batch", "2", "--seq", "128", "--bucket-mb", "1"],
            "llama-zero1": ["--model", "tiny", "--batch", "2", "--seq", "128", "--bucket-mb", "1", "--zero1"],
            "llama-fp32": ["--model", "tiny", "--batch", "2", "--seq", "128", "--bucket-mb", "1", "--grad-reduce", "fp32"],
            "mnist": ["--model", "mnist-cnn", "--batch", "64", "--graph", "off", "--dropout", "off"]}[case] + COMMON
    one = _run(args + ["--data-ranks", "2"])
    two = _run(args + ["--check-reduction"], port=29631 + ["llama", "llama-zero1", "llama-fp32", "mnist"].index(case))
    cr = two["check_reduction"]
    print(json.dumps({"case": case, "check_reduction": cr, "fp_two": two["update_fingerprint"],
                      "fp_one": one["update_fingerprint"]}))
    assert two["n_gpus"] == 2 and two["placement_source"] == "rehearsal"
    assert cr["ok"] and cr["world"] == 2 and cr["buckets"] >= 1, cr
    assert _rel(two["update_fingerprint"], one["update_fingerprint"]) < 2e-2
