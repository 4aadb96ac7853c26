"""Training checkpoints (models/checkpoint.py): async sharded save, exact resume, and resharding
across world sizes / ZeRO-1 settings.  CPU: single process and gloo at world_size 2 (127.0.0.1)."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
from safetensors import safe_open

from gpu_topology_on_k8s_amd.models import CheckpointWriter, FlatAdamW, Llama, LlamaConfig, load_checkpoint
from gpu_topology_on_k8s_amd.models.checkpoint import latest_checkpoint, read_optimizer_ranges, read_ranges


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _steps(m, opt, gen, n, cfg):
    for _ in range(n):
        tok = torch.randint(0, cfg.vocab, (2, 16), generator=gen)
        m.flat.zero_grad()
        m(tok, torch.roll(tok, -1, 1)).backward()
        opt.step()


def test_save_resume_single_process_is_exact(tmp_path):
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu", seed=1)
    opt = FlatAdamW(m.flat, lr=1e-3)
    gen = torch.Generator().manual_seed(5)
    _steps(m, opt, gen, 2, cfg)
    w = CheckpointWriter(str(tmp_path), m, opt, model_name="tiny")
    w.save(2, gen)
    w.close()
    _steps(m, opt, gen, 2, cfg)  # continuous run: steps 3, 4
    want = m.flat.data.clone()

    m2 = Llama(cfg, device="cpu", seed=99)  # different init: everything must come from the file
    opt2 = FlatAdamW(m2.flat, lr=1e-3)
    gen2 = torch.Generator().manual_seed(0)
    meta = load_checkpoint(str(tmp_path), m2, opt2, gen2)
    assert meta["step"] == 2 and opt2.t == 2 and meta["path"] == latest_checkpoint(str(tmp_path))
    _steps(m2, opt2, gen2, 2, cfg)
    assert torch.equal(m2.flat.data, want)


def test_keep_prunes_and_latest_points_at_newest(tmp_path):
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu")
    opt = FlatAdamW(m.flat)
    w = CheckpointWriter(str(tmp_path), m, opt, keep=2)
    for s in (1, 2, 3):
        w.save(s)
    w.close()
    dirs = sorted(d for d in os.listdir(tmp_path) if d.startswith("step_"))
    assert dirs == ["step_000002", "step_000003"]
    assert open(tmp_path / "latest").read() == "step_000003"
    assert not [d for d in os.listdir(tmp_path) if d.endswith(".tmp")]
    meta = json.load(open(tmp_path / "step_000003" / "meta.json"))
    assert meta["numel"] == m.flat.numel and meta["layout"][0][0] == m.flat.names[0]


def test_a_resumed_run_saving_older_steps_keeps_its_latest(tmp_path):
    """A run resumed from an older step writes lower step numbers than the directories left behind by
    the run it replaces: the step ``latest`` names is never the one pruned, and with keep = 1 it is the
    only one left."""
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu")
    opt = FlatAdamW(m.flat)
    w = CheckpointWriter(str(tmp_path), m, opt, keep=1)
    w.save(5)
    w.close()
    w = CheckpointWriter(str(tmp_path), m, opt, keep=1)  # resumed from an older step, saving step 3
    w.save(3)
    w.close()
    assert open(tmp_path / "latest").read() == "step_000003"
    assert sorted(d for d in os.listdir(tmp_path) if d.startswith("step_")) == ["step_000003"]
    assert latest_checkpoint(str(tmp_path)).endswith("step_000003")


def test_a_resumed_run_keeps_its_own_checkpoints_not_the_abandoned_runs(tmp_path):
    """ADVICE r5 (checkpoint.py:314): the abandoned run saved 100, 200 and 300; this run resumes from 100
    with keep = 2 and saves 150, then 250.  The survivors are this run's current step and its
    predecessor: the abandoned run's 200 and 300 are gone at the first save, so no later save deletes
    this run's previous checkpoint to keep them, and the fallback never picks them."""
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu")
    opt = FlatAdamW(m.flat)
    w = CheckpointWriter(str(tmp_path), m, opt, keep=3)
    for s in (100, 200, 300):
        w.save(s)
    w.close()
    w = CheckpointWriter(str(tmp_path), m, opt, keep=2)  # resumed from step 100
    w.save(150)
    w.close()
    assert sorted(d for d in os.listdir(tmp_path) if d.startswith("step_")) == ["step_000100", "step_000150"]
    w = CheckpointWriter(str(tmp_path), m, opt, keep=2)
    w.save(250)
    w.close()
    assert sorted(d for d in os.listdir(tmp_path) if d.startswith("step_")) == ["step_000150", "step_000250"]
    os.unlink(tmp_path / "step_000250" / "meta.json")  # latest names an incomplete directory: the fallback
    assert latest_checkpoint(str(tmp_path)).endswith("step_000150")  # finds this run's, not the old run's 300


def test_layout_mismatch_is_refused(tmp_path):
    m = Llama(LlamaConfig.tiny(), device="cpu")
    w = CheckpointWriter(str(tmp_path), m, FlatAdamW(m.flat))
    w.save(1)
    w.close()
    import dataclasses
    cfg = dataclasses.replace(LlamaConfig.tiny(), n_layers=3)
    other = Llama(cfg, device="cpu")
    with pytest.raises(ValueError, match="layout"):
        load_checkpoint(str(tmp_path), other, FlatAdamW(other.flat))
    with pytest.raises(FileNotFoundError):
        load_checkpoint(str(tmp_path / "nothing"), m)


def test_optimizer_ranges_reshard(tmp_path):
    """State written as 3 uneven shards reads back for any other tiling of the buffer."""
    n = 1000
    full = {k: torch.randn(n) for k in ("master", "m", "v")}
    shards = [[(0, 100), (700, 1000)], [(100, 450)], [(450, 700)]]
    from safetensors.torch import save_file
    for r, sh in enumerate(shards):
        t = {k: torch.cat([full[k][s:e] for s, e in sh]) for k in full}
        t["shards"] = torch.tensor(sh, dtype=torch.int64)
        save_file(t, str(tmp_path / f"state_rank{r}.safetensors"))
    for ranges in ([(0, n)], [(0, 500)], [(500, 1000)], [(50, 120), (600, 990)]):
        got = read_optimizer_ranges(str(tmp_path), ranges)
        for k in full:
            assert torch.equal(got[k], torch.cat([full[k][s:e] for s, e in ranges]))
    with pytest.raises(ValueError, match="cover"):
        read_optimizer_ranges(str(tmp_path), [(0, n + 10)])


def _worker(rank, world, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from gpu_topology_on_k8s_amd.models.train import train
    import torch.distributed as dist

    kw = dict(batch=2, seq=16, warmup=0, device_kind="cpu", log=False, zero1=True, bucket_mb=0.05)
    a = train("tiny", steps=4, save_dir=os.path.join(root, "a"), **kw)
    b1 = train("tiny", steps=2, save_dir=os.path.join(root, "b"), save_every=1, **kw)
    b2 = train("tiny", steps=2, save_dir=os.path.join(root, "b"), resume=os.path.join(root, "b"), **kw)
    # replicated (no ZeRO-1): each rank writes half of the state; resume is exact too
    kw["zero1"] = False
    train("tiny", steps=3, save_dir=os.path.join(root, "c"), **kw)
    train("tiny", steps=1, save_dir=os.path.join(root, "d"), **kw)
    train("tiny", steps=2, save_dir=os.path.join(root, "d"), resume=os.path.join(root, "d"), **kw)
    q.put((rank, {"a": a["step_end"], "b1": b1["checkpoints_saved"], "b2": (b2["step_start"], b2["step_end"]),
                  "loss_a": a["loss_last"], "loss_b": b2["loss_last"]}))
    dist.destroy_process_group()


def test_replicated_state_is_split_over_ranks(tmp_path):
    """Without ZeRO-1 every rank writes a 1/W slice (8-aligned) of weights and optimizer state."""
    m = Llama(LlamaConfig.tiny(), device="cpu")
    opt = FlatAdamW(m.flat)
    n = m.flat.numel
    spans = []
    for r in range(3):
        w = CheckpointWriter.__new__(CheckpointWriter)
        w.model, w.opt, w.rank, w.world = m, opt, r, 3
        spans += w.write_ranges()
    assert spans[0][0] == 0 and spans[-1][1] == n and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert all(s % 8 == 0 for s, _ in spans)


def test_zero1_two_ranks_resume_matches_continuous_and_reshards_to_one(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r]["a"] == 4 and res[r]["b1"] == [1, 2] and res[r]["b2"] == (2, 4)
        assert res[r]["loss_a"] == res[r]["loss_b"]
    da, db = latest_checkpoint(str(tmp_path / "a")), latest_checkpoint(str(tmp_path / "b"))
    assert da.endswith("step_000004") and db.endswith("step_000004")
    # each ZeRO-1 rank wrote only its own shard (weights and optimizer state)
    assert sorted(f for f in os.listdir(da) if f.startswith("state")) == ["state_rank0.safetensors", "state_rank1.safetensors"]
    numel = json.load(open(os.path.join(da, "meta.json")))["numel"]
    wa = read_ranges(da, [(0, numel)], ("flat",))["flat"]
    wb = read_ranges(db, [(0, numel)], ("flat",))["flat"]
    assert wa.dtype == torch.bfloat16 and torch.equal(wa, wb)  # resumed run == continuous run
    dc, dd = latest_checkpoint(str(tmp_path / "c")), latest_checkpoint(str(tmp_path / "d"))
    assert sorted(f for f in os.listdir(dc) if f.startswith("state")) == ["state_rank0.safetensors", "state_rank1.safetensors"]
    keys = ("flat", "master", "m", "v")
    sc, sd = read_ranges(dc, [(0, numel)], keys), read_ranges(dd, [(0, numel)], keys)
    assert all(torch.equal(sc[k], sd[k]) for k in keys)
    # reshard: the 2-rank ZeRO-1 state resumes into one unsharded optimizer (world 1)
    m = Llama(LlamaConfig.tiny(), device="cpu", seed=3)
    opt = FlatAdamW(m.flat)
    meta = load_checkpoint(da, m, opt)
    assert meta["world"] == 2 and meta["zero1"] and opt.t == 4
    for fn in ("state_rank0.safetensors", "state_rank1.safetensors"):
        with safe_open(os.path.join(da, fn), "pt") as f:
            o = 0
            master = f.get_tensor("master")
            for s, e in f.get_tensor("shards").tolist():
                assert torch.equal(opt.master[s:e], master[o:o + e - s])
                o += e - s


@pytest.mark.gpu
def test_async_checkpoint_on_gpu_resumes_exactly(tmp_path):
    """HIP path: pinned async snapshot on a side stream while the next steps run (fused AdamW
    kernel, HIP attention), then an exact resume into a fresh model on the device."""
    from gpu_topology_on_k8s_amd.ops import fused

    fused.hip()  # fail loudly if the extension is missing
    dev = torch.device("cuda", 0)
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device=dev, seed=1)
    opt = FlatAdamW(m.flat, lr=1e-3)
    gen = torch.Generator().manual_seed(5)

    def steps(m, opt, gen, n):
        for _ in range(n):
            tok = torch.randint(0, cfg.vocab, (2, 64), generator=gen).to(dev)
            m.flat.zero_grad()
            m(tok, torch.roll(tok, -1, 1)).backward()
            opt.step()

    steps(m, opt, gen, 2)
    snap = (m.flat.data.clone(), opt.master.clone(), opt.v.clone())
    w = CheckpointWriter(str(tmp_path), m, opt, model_name="tiny")
    w.save(2, gen)  # returns before the file is written
    steps(m, opt, gen, 2)  # these steps overwrite the state while the writer runs
    w.close()
    torch.cuda.synchronize()
    want = m.flat.data.clone()
    d = latest_checkpoint(str(tmp_path))
    st = read_ranges(d, [(0, m.flat.numel)], ("flat", "master", "v"))
    assert torch.equal(st["flat"], snap[0].cpu())  # the snapshot, not later state
    assert torch.equal(st["master"], snap[1].cpu()) and torch.equal(st["v"], snap[2].cpu())
    m2 = Llama(cfg, device=dev, seed=7)
    opt2 = FlatAdamW(m2.flat, lr=1e-3)
    gen2 = torch.Generator()
    load_checkpoint(str(tmp_path), m2, opt2, gen2)
    steps(m2, opt2, gen2, 2)
    torch.cuda.synchronize()
    assert torch.equal(m2.flat.data, want)


def test_latest_survives_crash_while_replacing_a_step(tmp_path):
    """re-saving an existing step moves it aside first; `latest` must never dangle."""
    import json as _json

    from gpu_topology_on_k8s_amd.models.checkpoint import latest_checkpoint

    root = tmp_path
    for s in (999999, 1000000):
        d = root / f"step_{s:06d}"
        d.mkdir()
        (d / "meta.json").write_text(_json.dumps({"step": s}))
    (root / "latest").write_text("step_1000000")
    assert latest_checkpoint(str(root)).endswith("step_1000000")
    (root / "step_1000000").rename(root / ".step_1000000.old")  # crash between the two renames
    assert latest_checkpoint(str(root)).endswith(".step_1000000.old")
    (root / ".step_1000000.old" / "meta.json").unlink()
    assert latest_checkpoint(str(root)).endswith("step_999999")  # numeric, not lexicographic


def test_stray_step_directories_are_ignored(tmp_path):
    """A directory named like a step but not one ("step_¹": a digit to str.isdigit, not to int) is
    neither resumed from nor pruned, and does not break either."""
    import os

    from gpu_topology_on_k8s_amd.models.checkpoint import latest_checkpoint

    os.makedirs(tmp_path / "step_¹")
    os.makedirs(tmp_path / "step_x")
    assert latest_checkpoint(str(tmp_path)) is None
