"""Llama workload on CPU: model math, flat parameter layout, fused-AdamW reference, and the bucketed
RCCL-style gradient all-reduce exercised with gloo at world_size 2 (multi-process, 127.0.0.1)."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpu_topology_on_k8s_amd.models import FlatAdamW, Llama, LlamaConfig
from gpu_topology_on_k8s_amd.ops import fused
from gpu_topology_on_k8s_amd.parallel.dp import BucketedAllReduce


def test_llama3_8b_config_matches_published_size():
    cfg = LlamaConfig.llama3_8b()
    assert cfg.head_dim == 128
    n = cfg.num_params()
    assert 8.0e9 < n < 8.1e9  # Llama-3-8B: 8.03 B parameters
    # 288 GB HBM budget: bf16 weights + bf16 grads + fp32 master/m/v
    assert n * (2 + 2 + 12) / 1e9 < 140


def test_flat_params_are_views_and_aligned():
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu")
    f = m.flat
    for n, p in f.params.items():
        o, e = f.span(n)
        assert p.data_ptr() == f.data[o:].data_ptr()
        assert p.grad.data_ptr() == f.grad[o:].data_ptr()
        assert o % 64 == 0
    assert f.numel >= cfg.num_params()


def test_forward_backward_accumulates_into_flat_grad():
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu")
    tok = torch.randint(0, cfg.vocab, (2, 32))
    loss = m(tok, torch.roll(tok, -1, 1))
    assert abs(loss.item() - math.log(cfg.vocab)) < 0.5  # random init ~ uniform prediction
    loss.backward()
    assert m.flat.grad.float().abs().sum() > 0
    assert all(p.grad.data_ptr() == m.flat.grad[m.flat.span(n)[0]:].data_ptr() for n, p in m.flat.params.items())


def test_direct_weight_grads_match_autograd_and_accumulate():
    """Projection weight gradients written in place by the GEMM (models/llama.py _FlatLinear) equal
    plain autograd's, a second backward without zero_grad accumulates, zero_grad restarts."""
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu", seed=3)
    assert "lm_head" in m.flat.direct and "l0.wqkv" in m.flat.direct and "tok_emb" not in m.flat.direct
    tok = torch.randint(0, cfg.vocab, (2, 16), generator=torch.Generator().manual_seed(5))
    lab = torch.roll(tok, -1, 1)
    m.flat.zero_grad()
    m(tok, lab).backward()
    g1 = m.flat.grad.float().clone()
    # reference: the same math with every weight an ordinary autograd leaf
    ref = {n: p.detach().float().clone().requires_grad_(True) for n, p in m.flat.params.items()}
    x = torch.nn.functional.embedding(tok.reshape(-1), ref["tok_emb"])
    B, S = tok.shape
    H, Hkv, Dh = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
    cos, sin = fused.rope_tables(cfg.max_seq, Dh, cfg.rope_theta)
    for i in range(cfg.n_layers):
        h = fused.rmsnorm_ref(x, ref[f"l{i}.attn_norm"], cfg.norm_eps)
        q, k, v = fused.rope_split_ref(h @ ref[f"l{i}.wqkv"].t(), cos, sin, B, S, H, Hkv, Dh)
        o = fused.attention_ref(q, k, v).reshape(B * S, H * Dh)
        x = x + o @ ref[f"l{i}.wo"].t()
        h = fused.rmsnorm_ref(x, ref[f"l{i}.ffn_norm"], cfg.norm_eps)
        x = x + fused.swiglu_ref(h @ ref[f"l{i}.w13"].t()) @ ref[f"l{i}.w2"].t()
    logits = fused.rmsnorm_ref(x, ref["norm"], cfg.norm_eps) @ ref["lm_head"].t()
    torch.nn.functional.cross_entropy(logits.float(), lab.reshape(-1)).backward()
    for n in ("lm_head", "l0.wqkv", "l1.w2", "l0.wo"):
        o_, e_ = m.flat.span(n)
        got, want = g1[o_:e_].view_as(ref[n]), ref[n].grad
        assert (got - want).norm() / want.norm() < 5e-2, n
    m(tok, lab).backward()  # no zero_grad: accumulate
    assert torch.allclose(m.flat.grad.float(), 2 * g1, rtol=2e-2, atol=1e-4)
    m.flat.zero_grad()
    m(tok, lab).backward()
    assert torch.allclose(m.flat.grad.float(), g1, rtol=1e-2, atol=1e-5)


def test_nt_gemm_layout_matches_native():
    """Backward GEMMs in NT layout (transposed operands) give the native layout's gradients."""
    cfg = LlamaConfig.tiny()
    tok = torch.randint(0, cfg.vocab, (2, 16), generator=torch.Generator().manual_seed(7))
    grads = {}
    for layout in ("native", "nt"):
        m = Llama(cfg, device="cpu", seed=3, gemm_layout=layout)
        m.flat.zero_grad()
        m(tok, torch.roll(tok, -1, 1)).backward()
        grads[layout] = m.flat.grad.float().clone()
    assert torch.allclose(grads["nt"], grads["native"], rtol=1e-2, atol=1e-5)
    with pytest.raises(ValueError):
        Llama(cfg, device="cpu", gemm_layout="tn")


def test_swiglu_bwd_ref_matches_autograd():
    gu = torch.randn(8, 64, dtype=torch.float64, requires_grad=True)
    dh = torch.randn(8, 32, dtype=torch.float64)
    fused.swiglu_ref(gu).backward(dh)
    assert torch.allclose(fused.swiglu_bwd_ref(dh, gu.detach()).double(), gu.grad, rtol=1e-5, atol=1e-6)
    dgu, dgu_t = fused.swiglu_bwd_t(dh, gu.detach())
    assert torch.equal(dgu_t, dgu.t().contiguous())


def test_reference_ops_match_definitions():
    x = torch.randn(4, 64, dtype=torch.bfloat16)
    w = torch.rand(64, dtype=torch.bfloat16) + 0.5
    y = fused.rmsnorm_ref(x, w, 1e-5).float()
    want = x.float() / torch.sqrt(x.float().pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    assert torch.allclose(y, want, atol=3e-2, rtol=2e-2)
    cos, sin = fused.rope_tables(16, 32)
    qkv = torch.randn(2 * 16, (4 + 2 * 2) * 32, dtype=torch.bfloat16)
    q, k, v = fused.rope_split_ref(qkv, cos, sin, 2, 16, 4, 2, 32)
    assert q.shape == (2, 4, 16, 32) and k.shape == (2, 2, 16, 32) and v.shape == (2, 2, 16, 32)
    # position 0 is the identity rotation
    assert torch.equal(q[:, :, 0], qkv.view(2, 16, 8, 32)[:, 0, :4])
    # rotation preserves norms
    assert torch.allclose(q.float().norm(dim=-1), qkv.view(2, 16, 8, 32)[:, :, :4].float().transpose(1, 2).norm(dim=-1), rtol=2e-2)


def test_flat_adamw_reference_matches_torch_adamw():
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu")
    ref = [p.detach().float().clone().requires_grad_(True) for p in m.flat.params.values()]
    topt = torch.optim.AdamW(ref, lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    opt = FlatAdamW(m.flat, lr=1e-3, weight_decay=0.1, clip_norm=None)
    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        m.flat.grad.copy_(torch.randn(m.flat.numel, generator=g).to(torch.bfloat16))
        for r, (n, p) in zip(ref, m.flat.params.items()):
            r.grad = p.grad.detach().float().clone()
        topt.step()
        opt.step()
    for r, (n, p) in zip(ref, m.flat.params.items()):
        o, e = m.flat.span(n)
        assert torch.allclose(opt.master[o:e].view_as(r), r.detach(), atol=1e-5, rtol=1e-4), n


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    cfg = LlamaConfig.tiny()
    m = Llama(cfg, device="cpu", seed=7)
    # tiny buckets so the model spans many of them and hooks fire in backward order
    ar = BucketedAllReduce(m.flat, bucket_mb=0.05, first_bucket_mb=0.01)
    opt = FlatAdamW(m.flat, lr=1e-3)
    gen = torch.Generator().manual_seed(100 + rank)  # different data per rank
    ref = Llama(cfg, device="cpu", seed=7)  # hook-free replica: the expected gradient, reduced separately
    out = {"buckets": len(ar.buckets)}
    for step in range(2):
        tok = torch.randint(0, cfg.vocab, (2, 16), generator=gen)
        m.flat.zero_grad()
        loss = m(tok, torch.roll(tok, -1, 1))
        loss.backward()  # buckets are all-reduced in place from the hooks while backward runs
        ar.finish()
        if step == 0:
            ref.flat.zero_grad()
            ref(tok, torch.roll(tok, -1, 1)).backward()
            want = ref.flat.grad.float()
            dist.all_reduce(want)
            out["allreduce_ok"] = bool(torch.allclose(m.flat.grad.float(), want, atol=2e-2, rtol=2e-2))
            out["launches"] = ar.stats["launches"]
        opt.step(grad_scale=ar.grad_scale)
    ck = m.flat.data.float().sum().item()
    t = torch.tensor([ck])
    gathered = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(gathered, t)
    out["replicas_equal"] = all(abs(g.item() - gathered[0].item()) < 1e-6 for g in gathered)
    # stragglers: buckets no backward hook launched (parameters that got no gradient) are launched by
    # finish() itself; here no backward runs at all, so finish() must reduce every bucket
    before = ar.stats["launches"]
    m.flat.grad.fill_(rank + 1)
    ar.finish()
    out["straggler_launches"] = ar.stats["launches"] - before
    out["stragglers_reduced"] = bool((m.flat.grad.float() == world * (world + 1) / 2).all())
    tiles = sorted((b.start, b.end) for b in ar.buckets)
    out["tiled"] = tiles[0][0] == 0 and tiles[-1][1] == m.flat.numel and all(a[1] == b[0] for a, b in zip(tiles, tiles[1:]))
    q.put((rank, out))
    dist.destroy_process_group()


def test_bucketed_allreduce_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r]["buckets"] > 3
        assert res[r]["allreduce_ok"], res
        assert res[r]["launches"] == res[r]["buckets"]  # every bucket launched from a backward hook
        assert res[r]["replicas_equal"]
        assert res[r]["tiled"]
        assert res[r]["straggler_launches"] == res[r]["buckets"] and res[r]["stragglers_reduced"], res[r]


def _zero1_worker(rank, world, port, q):
    """Same data, same seed: ZeRO-1 (reduce-scatter grads, sharded AdamW, async all-gather waited per
    bucket in the next forward) must track the all-reduce + full AdamW run step for step."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()
    runs = {}
    for zero1 in (False, True):
        m = Llama(cfg, device="cpu", seed=7)
        ar = BucketedAllReduce(m.flat, bucket_mb=0.05, first_bucket_mb=0.01, zero1=zero1)
        opt = FlatAdamW(m.flat, lr=1e-3, shards=ar.shards() if zero1 else None)
        if zero1:
            m.param_ready = ar.wait_param
        gen = torch.Generator().manual_seed(100 + rank)
        losses = []
        for _ in range(3):
            tok = torch.randint(0, cfg.vocab, (2, 16), generator=gen)
            m.flat.zero_grad()
            loss = m(tok, torch.roll(tok, -1, 1))
            loss.backward()
            ar.finish()
            opt.step(grad_scale=ar.grad_scale)
            ar.gather_params()
            losses.append(float(loss))
        ar.wait_all_params()
        runs[zero1] = (m.flat.data.float().clone(), losses, opt.master.numel(), len(ar.buckets))
        ar.remove()
    full, sharded = runs[False], runs[True]
    ck = torch.tensor([sharded[0].sum().item()])
    gathered = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(gathered, ck)
    q.put((rank, {
        "max_diff": float((full[0] - sharded[0]).abs().max()),
        "loss_diff": max(abs(a - b) for a, b in zip(full[1], sharded[1])),
        "state_ratio": sharded[2] / full[2],
        "buckets": sharded[3],
        "replicas_equal": all(abs(g.item() - gathered[0].item()) < 1e-6 for g in gathered),
    }))
    dist.destroy_process_group()


def test_zero1_matches_allreduce_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_zero1_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert res[r]["buckets"] > 3
        assert res[r]["state_ratio"] == pytest.approx(1 / world)
        assert res[r]["replicas_equal"], res
        assert res[r]["loss_diff"] < 1e-2, res
        assert res[r]["max_diff"] < 2e-2, res  # bf16 weights; reduction order differs (RS vs AR)


@pytest.mark.parametrize("zero1", [False, True])
def test_train_entry_cpu_single_rank(zero1):
    from gpu_topology_on_k8s_amd.models.train import train

    if dist.is_initialized():
        pytest.skip("process group already initialised")
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    try:
        out = train("tiny", batch=2, seq=32, steps=2, warmup=1, device_kind="cpu", log=False, zero1=zero1)
    finally:
        dist.destroy_process_group()
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
            os.environ.pop(k, None)
    assert out["tokens_per_s"] > 0 and out["steps"] == 2 and math.isfinite(out["loss_last"])
    assert out["zero1"] == zero1 and out["optimizer_state_gb"] > 0


def test_train_repeat_batch_memorises():
    """--repeat-batch: one batch at every step must be learnt (forward, backward and AdamW end to end);
    the same run on the GPU at the Llama-3-8B shape is profiles/r03_learn/."""
    from gpu_topology_on_k8s_amd.models.train import train

    if dist.is_initialized():
        pytest.skip("process group already initialised")
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    try:
        out = train("tiny", batch=2, seq=32, steps=25, warmup=0, device_kind="cpu", log=False, lr=3e-3,
                    repeat_batch=True)
    finally:
        dist.destroy_process_group()
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
            os.environ.pop(k, None)
    losses = out["losses"]
    assert out["repeat_batch"] and len(losses) == 25
    assert losses[-1] < 0.5 * losses[0], losses


def test_best_vs_worst_harness_cpu_dry_run(tmp_path):
    """bench/train_llama.py (BASELINE config 5 / Gaia Exp. 6) end to end on CPU: two 2-rank gloo jobs
    placed on a fake 8-device node, best and worst being different real device sets (k < n)."""
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "r.json"
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(repo, "bench", "train_llama.py"), "--gpus", "2", "--device", "cpu",
                        "--discovery", "fake", "--model", "tiny", "--batch", "1", "--seq", "64", "--steps", "2", "--warmup", "1",
                        "--attn", "sdpa", "--gemm-tuning", "off", "--out", str(out)],
                       capture_output=True, text=True, timeout=600, cwd=repo, env=dict(env, GTK_FAKE_GPUS="8"))
    assert p.returncode == 0, p.stderr[-4000:]
    s = json.loads(out.read_text())["summary"]
    assert s["worst_kind"] == "worst" and s["best_devices"] != s["worst_devices"]
    assert len(s["best_devices"]) == 2 and s["best_tokens_per_s"] > 0 and s["worst_tokens_per_s"] > 0
    assert s["best_score"] > s["worst_score"]


def _reduce_dtype_worker(rank, world, port, q):
    """Different data per rank: the gradient each reduction delivers against the exact (float64) sum of
    the ranks' local gradients."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = LlamaConfig.tiny()
    tok = torch.randint(0, cfg.vocab, (2, 32), generator=torch.Generator().manual_seed(200 + rank))
    ref = Llama(cfg, device="cpu", seed=7)  # hook-free replica: this rank's local gradient
    ref.flat.zero_grad()
    ref(tok, torch.roll(tok, -1, 1)).backward()
    local = ref.flat.grad.double()
    parts = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(parts, local)
    exact = torch.stack(parts).sum(0)
    out = {}
    for mode in ("bf16", "fp32"):
        m = Llama(cfg, device="cpu", seed=7)
        ar = BucketedAllReduce(m.flat, bucket_mb=0.05, first_bucket_mb=0.01, grad_reduce=mode)
        m.flat.zero_grad()
        m(tok, torch.roll(tok, -1, 1)).backward()
        ar.finish()
        got = (ar.reduced_grad if ar.reduced_grad is not None else m.flat.grad).double()
        out[mode] = float((got - exact).norm() / exact.norm())
        # the averaged gradient the optimizer applies (sum x grad_scale) against the exact average
        out[mode + "_avg"] = float((got * ar.grad_scale - exact / world).norm() / (exact / world).norm())
        out[mode + "_dtype"] = str(got.dtype if ar.reduced_grad is None else ar.reduced_grad.dtype)
        ar.remove()
    q.put((rank, out))
    dist.destroy_process_group()


def test_fp32_gradient_reduction_matches_the_exact_sum_four_ranks_gloo():
    """4 ranks, different batches: the fp32 reduction's averaged gradient is within 1e-3 (relative norm)
    of the exact average of the ranks' local gradients; the bf16 in-place reduction's error is reported
    (it rounds every partial sum to bf16)."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_reduce_dtype_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    print({r: {k: res[r][k] for k in ("bf16", "fp32")} for r in res})
    for r in range(world):
        assert res[r]["fp32"] <= 1e-3 and res[r]["fp32_avg"] <= 1e-3, res[r]
        assert res[r]["fp32"] < res[r]["bf16"], res[r]  # the bf16 ring rounds; fp32 does not
        assert res[r]["bf16"] < 2e-2, res[r]
        assert res[r]["fp32_dtype"] == "torch.float32"


def test_transposed_gradient_hand_off_matches_only_the_same_tensor():
    """ops/fused.py offer_t / take_t: a consumer gets the offered transpose only for the very gradient
    it was offered for (storage, shape, strides and version), once; anything else falls back."""
    from gpu_topology_on_k8s_amd.ops import fused

    g = torch.randn(8, 4)
    gt = g.t().contiguous()
    fused.offer_t(g, gt)
    assert fused.take_t(torch.randn(8, 4)) is None  # another tensor
    assert fused.take_t(g) is gt
    assert fused.take_t(g) is None  # taken once
    fused.offer_t(g, gt)
    g.add_(1.0)  # modified after the offer: the transpose is stale
    assert fused.take_t(g) is None
    fused.offer_t(g, gt)
    assert fused.take_t(g.view(4, 8)) is None  # other shape
    fused.clear_t()
    assert not fused._PENDING_T
