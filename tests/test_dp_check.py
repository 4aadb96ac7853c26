"""The data-parallel correctness checks can fail.

``models/train.py --check-reduction`` and the SGD update fingerprint are what the k >= 2 GPU tests
(tests/test_gpu_multi.py, tests/test_gpu_rehearsal.py) assert on.  Here, on CPU with gloo at world 2
and different data per rank, each check is shown to pass on the real reduction AND to fail on a
mutated one:

* one bucket's collective skipped (the rank applies its local gradient for that bucket);
* ``b.work.wait()`` removed from :meth:`BucketedAllReduce.finish` while the collectives are slow (a
  FIFO worker thread runs each one 0.05 s late on a side gloo group, so the optimizer-side read comes
  before the reduction lands; the check freezes the buffer at that read, before its own collectives);
* the same slow collectives WITH the wait: the check passes, so it is the missing wait it catches.

The SGD fingerprint of a 2-rank run must match a 1-rank run on the concatenated batch
(``--data-ranks 2``), and must not match when a bucket is skipped.
"""
import os
import queue
import socket
import threading
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

KW = dict(batch=2, seq=64, steps=1, warmup=1, device_kind="cpu", attn="sdpa", gemm_tuning="off", bucket_mb=0.05,
          log=False, optimizer="sgd", lr=0.5, fingerprint=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Done:
    def wait(self):
        return True


class _SlowDist:
    """``torch.distributed`` with every ``all_reduce`` run late, in issue order, by one worker thread
    on a side group (the main thread keeps the default group for everything else)."""

    def __init__(self, real, side):
        self._real, self._side = real, side
        self._q = queue.Queue()
        threading.Thread(target=self._loop, daemon=True).start()

    def __getattr__(self, name):
        return getattr(self._real, name)

    def _loop(self):
        while True:
            t, ev = self._q.get()
            time.sleep(0.05)
            self._real.all_reduce(t, group=self._side)
            ev.set()
            self._q.task_done()

    def all_reduce(self, t, group=None, async_op=False, **kw):
        ev = threading.Event()
        self._q.put((t, ev))
        w = type("SlowWork", (), {"wait": lambda self_: ev.wait()})()
        if async_op:
            return w
        w.wait()
        return None

    def drain(self):
        self._q.join()


def _worker(rank, world, port, mode, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpu_topology_on_k8s_amd.models.train import train
    from gpu_topology_on_k8s_amd.parallel import dp

    slow = None
    if mode == "skip_bucket":
        real_launch = dp.BucketedAllReduce._launch

        def launch(self, b):
            if b.index == 2:  # this bucket's collective never runs
                self._launched[b.index] = True
                b.work = _Done()
                return
            real_launch(self, b)

        dp.BucketedAllReduce._launch = launch
    if mode in ("slow", "slow_nowait"):
        side = dist.new_group(backend="gloo")
        slow = _SlowDist(dist, side)
        dp.dist = slow
    if mode == "slow_nowait":
        def finish(self):
            if hasattr(self.flat, "fill_unwritten"):
                self.flat.fill_unwritten()
            for b in self.buckets:
                if b.work is None:
                    self._launch(b)
            self.reset()  # ... and no b.work.wait()

        dp.BucketedAllReduce.finish = finish
    try:
        out = train("tiny", check_reduction=world > 1, data_ranks=2 if world == 1 else 0, **KW)
        if slow is not None:
            slow.drain()
        q.put((rank, {"check": out["check_reduction"], "fp": out["update_fingerprint"], "buckets": out["buckets"]}))
    finally:
        dist.destroy_process_group()


def _run(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _rel(a, b):
    return float(torch.tensor(a, dtype=torch.float64).sub(torch.tensor(b, dtype=torch.float64)).norm()
                 / torch.tensor(b, dtype=torch.float64).norm())


@pytest.fixture(scope="module")
def one_rank_concat():
    return _run("ok", world=1)[0]["fp"]


def test_reduction_check_passes_and_sgd_matches_the_concatenated_batch(one_rank_concat):
    res = _run("ok")
    for r in (0, 1):
        c = res[r]["check"]
        assert c["ok"] and c["world"] == 2 and c["buckets"] > 3, c
        assert c["reduce_max_rel"] <= 1e-2 and c["ready_max_rel"] <= 1e-2, c
    assert res[0]["fp"] == res[1]["fp"]  # all-reduced: every rank reports the same fingerprint
    assert _rel(res[0]["fp"], one_rank_concat) < 2e-2, (res[0]["fp"], one_rank_concat)


def test_a_skipped_bucket_fails_the_reduction_check_and_the_sgd_parity(one_rank_concat):
    res = _run("skip_bucket")
    for r in (0, 1):
        c = res[r]["check"]
        assert not c["ok"] and c["worst_bucket"] == 2 and c["reduce_max_rel"] > 0.1, c
    assert _rel(res[0]["fp"], one_rank_concat) > 5e-2, (res[0]["fp"], one_rank_concat)


def test_slow_collectives_pass_with_the_wait():
    res = _run("slow")
    for r in (0, 1):
        assert res[r]["check"]["ok"], res[r]["check"]


def test_a_missing_wait_fails_the_reduction_check():
    res = _run("slow_nowait")
    for r in (0, 1):
        c = res[r]["check"]
        assert not c["ok"] and c["reduce_max_rel"] > 0.1, c


def test_comm_ctas_auto_times_each_cap_and_keeps_the_fastest():
    """--comm-ctas auto (the default) at world > 1: after the warmup one
    communicator per candidate cap, two timed forward + backward + reduction passes each, the fastest
    kept and the table reported; the reduction check still holds across the switch of communicators
    (ZeRO-1 included).  The parity tests above run with the default too: the tuning passes leave the
    training itself unchanged."""
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "-m", "gpu_topology_on_k8s_amd.models.train",
                        "--model", "tiny", "--batch", "2", "--seq", "64", "--steps", "2", "--warmup", "1", "--device", "cpu",
                        "--attn", "sdpa", "--gemm-tuning", "off", "--bucket-mb", "0.05", "--zero1", "--check-reduction"],
                       capture_output=True, text=True, timeout=600, cwd=repo, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    table = out["comm_ctas_tuning"]
    from gpu_topology_on_k8s_amd.models.train import AUTO_CTAS

    assert [r["ctas"] for r in table] == list(AUTO_CTAS) and all(r["ms_per_pass"] > 0 for r in table)
    assert out["comm_ctas"] == min(table, key=lambda r: r["ms_per_pass"])["ctas"]
    assert out["check_reduction"]["ok"]
