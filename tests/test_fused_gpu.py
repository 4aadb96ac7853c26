"""HIP fused kernels vs plain PyTorch fp32 references (run on a real MI355X: ``pytest -m gpu``)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    assert torch.cuda.is_available(), "needs a GPU"
    from gpu_topology_on_k8s_amd.ops.fused import hip as load_hip

    return load_hip()  # raises (fails loudly) if the extension is missing


def fused_swiglu_bwd_ref(dh, gu):
    from gpu_topology_on_k8s_amd.ops.fused import swiglu_bwd_ref

    return swiglu_bwd_ref(dh.cpu(), gu.cpu()).cuda()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,D", [(1, 4096), (37, 4096), (513, 4096), (64, 2048), (33, 1000), (8, 8192)])
def test_rmsnorm_fwd_bwd(hip, M, D):
    torch.manual_seed(0)
    x = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    w = (torch.rand(D, device="cuda") + 0.5).to(torch.bfloat16)
    dy = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    y, rstd = hip.rmsnorm_fwd(x, w, 1e-5)
    xf, wf = x.float().requires_grad_(True), w.float().requires_grad_(True)
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    assert _rel(y, ref) < 5e-3
    ref.backward(dy.float())
    dx, dw = hip.rmsnorm_bwd(dy, x, w, rstd)
    assert _rel(dx, xf.grad) < 1e-2
    assert _rel(dw, wf.grad) < 1e-2


@pytest.mark.parametrize("M,D", [(1, 4096), (513, 4096), (33, 1000), (8, 8192)])
def test_add_rmsnorm_fwd_bwd(hip, M, D):
    """Fused residual add + RMSNorm vs fp32 autograd of h = x + r, y = rmsnorm(h) * w, with a
    gradient arriving on both outputs (dh from the residual stream, dy from the branch)."""
    torch.manual_seed(2)
    x = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    w = (torch.rand(D, device="cuda") + 0.5).to(torch.bfloat16)
    dy = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    dh = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    h, y, rstd = hip.add_rmsnorm_fwd(x, r, w, 1e-5)
    assert torch.equal(h, x + r)  # bf16 residual stream, bit-identical to the separate add
    xf, rf, wf = (t.float().requires_grad_(True) for t in (x, r, w))
    hf = xf + rf
    ref = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * wf
    assert _rel(y, ref) < 5e-3
    torch.autograd.backward([ref, hf], [dy.float(), dh.float()])
    dx, dw = hip.add_rmsnorm_bwd(dy, h, w, rstd, dh)
    assert _rel(dx, xf.grad) < 1e-2 and torch.equal(xf.grad, rf.grad)
    assert _rel(dw, wf.grad) < 1e-2


def test_rmsnorm_weight_grad_is_deterministic(hip):
    """dW is reduced in a fixed order (no atomics): bit-identical launch to launch at the Llama-3-8B
    shape [16384, 4096], and exact against an fp64 column sum of the same bf16 operands to bf16 rounding."""
    torch.manual_seed(3)
    M, D = 16384, 4096
    x = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    w = (torch.rand(D, device="cuda") + 0.5).to(torch.bfloat16)
    dy = torch.randn(M, D, device="cuda", dtype=torch.bfloat16)
    _, rstd = hip.rmsnorm_fwd(x, w, 1e-5)
    dws = [hip.rmsnorm_bwd(dy, x, w, rstd)[1] for _ in range(3)]
    assert all(torch.equal(dws[0], d) for d in dws[1:])
    ref = (dy.double() * x.double() * rstd.double()[:, None]).sum(0)
    assert _rel(dws[0], ref) < 4e-3


def test_llama_fused_residual_matches_unfused_gpu():
    """Whole tiny model: add+RMSNorm in one kernel (default) vs separate adds — same loss and
    gradients to bf16 rounding."""
    from gpu_topology_on_k8s_amd.models import Llama, LlamaConfig

    cfg = LlamaConfig.tiny()
    tok = torch.randint(0, cfg.vocab, (2, 128), device="cuda")
    out = {}
    for fuse in (False, True):
        m = Llama(cfg, device="cuda", seed=3, fuse_residual=fuse)
        m.flat.zero_grad()
        loss = m(tok, torch.roll(tok, -1, 1))
        loss.backward()
        out[fuse] = (loss.item(), m.flat.grad.float().clone())
    assert abs(out[True][0] - out[False][0]) < 1e-3
    assert _rel(out[True][1], out[False][1]) < 1e-2


@pytest.mark.parametrize("B,S,H,Hkv,Dh", [(2, 128, 32, 8, 128), (1, 77, 4, 2, 64), (1, 16, 8, 8, 32)])
def test_rope_split_fwd_bwd(hip, B, S, H, Hkv, Dh):
    from gpu_topology_on_k8s_amd.ops.fused import rope_split_ref, rope_tables

    torch.manual_seed(1)
    cos, sin = rope_tables(S + 8, Dh, device="cuda")
    qkv = torch.randn(B * S, (H + 2 * Hkv) * Dh, device="cuda", dtype=torch.bfloat16)
    q, k, v = hip.rope_split_fwd(qkv, cos, sin, B, S, H, Hkv, Dh, 0)
    qr, kr, vr = rope_split_ref(qkv.float(), cos, sin, B, S, H, Hkv, Dh)
    assert _rel(q, qr) < 5e-3 and _rel(k, kr) < 5e-3 and torch.equal(v, vr.to(torch.bfloat16))
    # backward == autograd of the fp32 reference
    x = qkv.float().requires_grad_(True)
    outs = rope_split_ref(x, cos, sin, B, S, H, Hkv, Dh)
    gs = [torch.randn_like(o) for o in outs]
    torch.autograd.backward(outs, gs)
    dqkv = hip.rope_split_bwd(*(g.to(torch.bfloat16).contiguous() for g in gs), cos, sin, 0)
    assert _rel(dqkv, x.grad) < 1e-2
    # offset positions
    q2, _, _ = hip.rope_split_fwd(qkv, cos, sin, B, S, H, Hkv, Dh, 8)
    q2r, _, _ = rope_split_ref(qkv.float(), cos, sin, B, S, H, Hkv, Dh, 8)
    assert _rel(q2, q2r) < 5e-3


@pytest.mark.parametrize("T,F", [(1, 14336), (300, 14336), (17, 64)])
def test_swiglu_fwd_bwd(hip, T, F):
    torch.manual_seed(2)
    gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    dh = torch.randn(T, F, device="cuda", dtype=torch.bfloat16)
    x = gu.float().requires_grad_(True)
    g, u = x.chunk(2, dim=-1)
    ref = torch.nn.functional.silu(g) * u
    assert _rel(hip.swiglu_fwd(gu), ref) < 5e-3
    ref.backward(dh.float())
    assert _rel(hip.swiglu_bwd(dh, gu), x.grad) < 1e-2


@pytest.mark.parametrize("T,V", [(5, 128256), (64, 1024), (3, 8)])
def test_cross_entropy_fwd_bwd(hip, T, V):
    torch.manual_seed(3)
    logits = (torch.randn(T, V, device="cuda") * 3).to(torch.bfloat16)
    labels = torch.randint(0, V, (T,), device="cuda")
    labels[0] = -100  # ignored row
    loss_rows, lse = hip.xent_fwd(logits, labels, -100)
    x = logits.float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(x, labels, ignore_index=-100, reduction="none")
    assert torch.allclose(loss_rows, ref, atol=2e-3, rtol=2e-3)
    assert torch.allclose(lse, torch.logsumexp(logits.float(), -1), atol=1e-3, rtol=1e-4)
    nvalid = (labels != -100).sum()
    ref.sum().div(nvalid).backward()
    g = logits.clone()
    hip.xent_bwd_inplace(g, labels, lse, (1.0 / nvalid.float()).reshape(1), -100)
    assert _rel(g, x.grad) < 1e-2
    assert g[0].float().abs().max() == 0  # ignored row has zero gradient


def test_cross_entropy_autograd_mean(hip):
    from gpu_topology_on_k8s_amd.ops.fused import cross_entropy

    torch.manual_seed(4)
    base = torch.randn(32, 4096, device="cuda")
    labels = torch.randint(0, 4096, (32,), device="cuda")
    a = base.to(torch.bfloat16).requires_grad_(True)
    la = cross_entropy(a * 1, labels)
    la.backward()
    b = base.to(torch.bfloat16).float().requires_grad_(True)
    lb = torch.nn.functional.cross_entropy(b, labels)
    lb.backward()
    assert abs(la.item() - lb.item()) < 1e-3
    assert _rel(a.grad, b.grad) < 1e-2


def test_adamw_and_sqnorm(hip):
    torch.manual_seed(5)
    n = 1 << 20
    master = torch.randn(n, device="cuda")
    m = torch.randn(n, device="cuda").abs() * 0.01
    v = torch.randn(n, device="cuda").abs() * 0.001
    g = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    w = master.to(torch.bfloat16)
    lr, b1, b2, eps, wd, gs, t = 1e-3, 0.9, 0.95, 1e-8, 0.1, 0.5, 3
    hp = torch.tensor([lr, b1, b2, eps, wd, gs, 1 - b1 ** t, 1 - b2 ** t], device="cuda")
    rm, rv, rp = m.clone(), v.clone(), master.clone()
    gg = g.float() * gs
    rm.mul_(b1).add_(gg, alpha=1 - b1)
    rv.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    rp -= lr * ((rm / (1 - b1 ** t)) / ((rv / (1 - b2 ** t)).sqrt() + eps) + wd * rp)
    hip.adamw_step(master, m, v, g, w, hp)
    assert torch.allclose(m, rm, atol=1e-6, rtol=1e-5) and torch.allclose(v, rv, atol=1e-7, rtol=1e-5)
    assert torch.allclose(master, rp, atol=1e-6, rtol=1e-5)
    assert torch.equal(w, rp.to(torch.bfloat16))
    sq = hip.sq_norm(g)
    assert math.isclose(sq.item(), g.float().pow(2).sum().item(), rel_tol=1e-4)


def test_sharded_flat_adamw_matches_full_on_gpu():
    """ZeRO-1 optimizer on the HIP kernels: per-shard launches on 8-element-aligned slices of the
    flat buffers (the ranges rank 1 of 4 owns) give bit-identical results to the full update."""
    from types import SimpleNamespace

    from gpu_topology_on_k8s_amd.models.optim import FlatAdamW

    torch.manual_seed(6)
    n = 64 * 1000
    data = torch.randn(n, device="cuda").to(torch.bfloat16)
    grad = torch.randn(n, device="cuda", dtype=torch.bfloat16)
    bounds = [0, 6400, 19200, 44800, n]  # bucket edges (multiples of 64)
    shards = []
    for s, e in zip(bounds, bounds[1:]):
        c = (e - s) // 4
        shards.append((s + c, s + 2 * c))
    full = FlatAdamW(SimpleNamespace(data=data.clone(), grad=grad, numel=n), lr=1e-3)
    part = FlatAdamW(SimpleNamespace(data=data.clone(), grad=grad, numel=n), lr=1e-3, clip_norm=None, shards=shards)
    full.clip_norm = None
    for _ in range(2):
        full.step(grad_scale=0.5)
        part.step(grad_scale=0.5)
    for s, e in shards:
        assert torch.equal(part.flat.data[s:e], full.flat.data[s:e])
    untouched = torch.ones(n, dtype=torch.bool, device="cuda")
    for s, e in shards:
        untouched[s:e] = False
    assert torch.equal(part.flat.data[untouched], data[untouched])
    assert part.state_bytes() * 4 == full.state_bytes()


@pytest.mark.parametrize("R,C", [(64, 64), (128, 4096), (4096, 192), (192, 384), (16384, 6144), (640, 128256)])
def test_transpose_kernel_exact(hip, R, C):
    x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
    y = hip.transpose_bf16(x)
    assert y.shape == (C, R) and torch.equal(y, x.t().contiguous())


@pytest.mark.parametrize("T,F", [(64, 64), (192, 128), (256, 14336), (4096, 192), (64, 384), (16384, 256)])
def test_swiglu_bwd_t_matches_bwd_and_transpose(hip, T, F):
    gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    dh = torch.randn(T, F, device="cuda", dtype=torch.bfloat16)
    dgu, dgu_t = hip.swiglu_bwd_t(dh, gu)
    ref = hip.swiglu_bwd(dh, gu)  # same math; allow a rare 1-ulp difference from FMA contraction
    assert (dgu.float() - ref.float()).abs().max().item() <= 1e-2 * ref.float().abs().max().item()
    assert _rel(dgu, fused_swiglu_bwd_ref(dh, gu)) < 1e-2
    assert dgu_t.shape == (2 * F, T) and torch.equal(dgu_t, dgu.t().contiguous())


def test_transpose_wrapper_fallback_shapes():
    from gpu_topology_on_k8s_amd.ops import fused

    x = torch.randn(100, 72, device="cuda", dtype=torch.bfloat16)  # not multiples of 64: torch copy
    assert torch.equal(fused.transpose(x), x.t().contiguous())


def test_llama_nt_layout_matches_native_gpu():
    """NT backward GEMMs (HIP transposes + hipBLASLt NT) vs the native layout on the GPU."""
    from gpu_topology_on_k8s_amd.models import Llama, LlamaConfig

    cfg = LlamaConfig.tiny()
    tok = torch.randint(0, cfg.vocab, (2, 128), device="cuda")
    grads = {}
    for layout, overlap in (("native", False), ("nt", False), ("nt", True)):
        m = Llama(cfg, device="cuda", seed=3, gemm_layout=layout, overlap_transposes=overlap)
        for _ in range(2):  # a weight update between steps: the side stream must see the new weights
            m.flat.zero_grad()
            m(tok, torch.roll(tok, -1, 1)).backward()
            with torch.no_grad():
                m.flat.data.add_(m.flat.grad, alpha=-1e-2)
        grads[(layout, overlap)] = m.flat.grad.float().clone()
    assert _rel(grads[("nt", False)], grads[("native", False)]) < 1e-2
    assert torch.equal(grads[("nt", True)], grads[("nt", False)])  # same kernels, only the stream differs
    m = Llama(cfg, device="cuda", seed=3, gemm_layout="nt", dgrad_nn=("wqkv", "wo", "w13", "w2", "lm_head"))
    for _ in range(2):
        m.flat.zero_grad()
        m(tok, torch.roll(tok, -1, 1)).backward()
        with torch.no_grad():
            m.flat.data.add_(m.flat.grad, alpha=-1e-2)
    assert _rel(m.flat.grad.float(), grads[("native", False)]) < 1e-2  # NN input gradients, NT weight gradients


def test_llama_model_gpu_matches_cpu_reference():
    """Full tiny model: HIP kernels + hipBLASLt on GPU vs the PyTorch reference path on CPU."""
    from gpu_topology_on_k8s_amd.models import Llama, LlamaConfig

    cfg = LlamaConfig.tiny()
    gm = Llama(cfg, device="cuda", seed=3)
    cm = Llama(cfg, device="cpu", seed=3)
    cm.flat.data.copy_(gm.flat.data.cpu())
    tok = torch.randint(0, cfg.vocab, (2, 64))
    lg = gm(tok.cuda(), torch.roll(tok, -1, 1).cuda())
    lc = cm(tok, torch.roll(tok, -1, 1))
    assert abs(lg.item() - lc.item()) < 2e-2
    lg.backward()
    lc.backward()
    assert _rel(gm.flat.grad.cpu(), cm.flat.grad) < 5e-2


def test_smoke_step_and_training_gpu():
    from gpu_topology_on_k8s_amd.models.llama import smoke_step

    assert math.isfinite(smoke_step("cuda:0"))


def test_overlapped_bucket_norm_matches_direct_gpu():
    """Per-bucket squared norms computed on a side stream as buckets complete (parallel/dp.py
    overlap_norm, installed even at world 1) equal the serial norm of the whole gradient, and a
    clipped AdamW step fed with them matches the one that computes the norm itself."""
    from gpu_topology_on_k8s_amd.models import FlatAdamW, Llama, LlamaConfig
    from gpu_topology_on_k8s_amd.parallel.dp import BucketedAllReduce

    cfg = LlamaConfig.tiny()
    tok = torch.randint(0, cfg.vocab, (2, 128), device="cuda")
    res = {}
    for overlap in (True, False):
        m = Llama(cfg, device="cuda", seed=3)
        ar = BucketedAllReduce(m.flat, bucket_mb=0.05, first_bucket_mb=0.01, overlap_norm=overlap)
        opt = FlatAdamW(m.flat, lr=1e-3, clip_norm=0.1)  # small clip: the norm decides the step
        for _ in range(2):
            m.flat.zero_grad()
            m(tok, torch.roll(tok, -1, 1)).backward()
            ar.finish()
            sq = ar.sq_norm()
            if overlap:
                assert sq is not None and len(ar.buckets) > 3
                want = m.flat.grad.float().pow(2).sum()
                assert abs(sq.item() - want.item()) <= 1e-4 * want.item()
            else:
                assert sq is None
            opt.step(grad_scale=ar.grad_scale, sq=sq)
        torch.cuda.synchronize()
        res[overlap] = m.flat.data.float().clone()
        ar.remove()
    assert _rel(res[True], res[False]) < 1e-3
