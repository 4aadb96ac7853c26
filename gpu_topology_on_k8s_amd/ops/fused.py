"""Autograd front-end of the fused HIP kernels (``csrc/ops/fused_ops.hip``) + PyTorch references.

GPU tensors always take the HIP path and fail loudly (``NativeUnavailable``) when the extension is
missing; CPU tensors take the reference path (used by the CPU test-suite and as the fp32 numerics
oracle of ``tests/test_fused_gpu.py``).
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from .._native import load

__all__ = [
    "rmsnorm", "rmsnorm_ref", "rope_tables", "rope_split", "rope_split_ref", "swiglu", "swiglu_ref", "cross_entropy",
    "cross_entropy_ref", "hip", "attention", "attention_ref", "flash_attention_supported", "transpose", "swiglu_bwd_ref",
    "swiglu_bwd_t", "swiglu_fwd_t", "attention_t", "offer_t", "take_t", "clear_t",
]


def hip():
    return load("_fused")


# ------------------------------------------------------------------------------------ transpose
def transpose(x: torch.Tensor) -> torch.Tensor:
    """Contiguous ``x.t()``: the LDS-tiled HIP kernel for bf16 GPU matrices whose dims are multiples of
    64 (every Llama-3 dim), torch's copy otherwise.  Puts backward-GEMM operands into the NT layout."""
    if x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.size(0) % 64 == 0 and x.size(1) % 64 == 0:
        return hip().transpose_bf16(x.contiguous())
    return x.t().contiguous()


# ----------------------------------------------------------------- transposed gradients, handed on
# A backward kernel that already holds a gradient tile in LDS can write the gradient's transpose too
# (xent_bwd_t: dlogits^T), which the consumer's NT-layout weight-gradient GEMM needs.  Autograd passes
# only the gradient itself between nodes, so the producer offers the transpose here, keyed by the
# gradient's storage, shape and version, and the consuming linear layer takes it (models/llama.py
# _FlatLinear).  The entry holds the gradient alive, so its address cannot be reused while the entry
# exists; a gradient that autograd summed or copied on the way has another address and simply finds
# nothing (the consumer transposes it itself).  Llama.forward clears leftovers.
_PENDING_T: Dict[Tuple[int, Tuple[int, ...]], Tuple[torch.Tensor, torch.Tensor, int]] = {}


def offer_t(g: torch.Tensor, g_t: torch.Tensor) -> None:
    _PENDING_T[(g.data_ptr(), tuple(g.shape))] = (g, g_t, g._version)


def take_t(g: torch.Tensor) -> Optional[torch.Tensor]:
    """The transpose a producer offered for exactly this gradient (same storage, shape, version), or None."""
    if not _PENDING_T:
        return None
    e = _PENDING_T.pop((g.data_ptr(), tuple(g.shape)), None)
    if e is None or e[2] != g._version or e[0].stride() != g.stride():
        return None
    return e[1]


def clear_t() -> None:
    _PENDING_T.clear()


# ------------------------------------------------------------------------------------ RMSNorm
def rmsnorm_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        x = x.contiguous()
        y, rstd = hip().rmsnorm_fwd(x, w, float(eps))
        ctx.save_for_backward(x, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dx, dw = hip().rmsnorm_bwd(dy.contiguous(), x, w, rstd)
        return dx, dw, None


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if x.is_cuda:
        return _RMSNorm.apply(x, w, eps)
    return rmsnorm_ref(x, w, eps)


class _AddRMSNorm(torch.autograd.Function):
    """``h = x + r; y = rmsnorm(h) * w`` as one node: the residual add lives in the norm kernel
    (forward) and the residual-stream gradient is accumulated inside the norm's backward kernel."""

    @staticmethod
    def forward(ctx, x, r, w, eps):
        h, y, rstd = hip().add_rmsnorm_fwd(x.contiguous(), r.contiguous(), w, float(eps))
        ctx.save_for_backward(h, w, rstd)
        return h, y

    @staticmethod
    def backward(ctx, dh, dy):
        h, w, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(h)
        if dh is None:
            dx, dw = hip().rmsnorm_bwd(dy.contiguous(), h, w, rstd)
        else:
            dx, dw = hip().add_rmsnorm_bwd(dy.contiguous(), h, w, rstd, dh.contiguous())
        return dx, dx, dw, None


def add_rmsnorm_ref(x: torch.Tensor, r: torch.Tensor, w: torch.Tensor, eps: float):
    h = x + r
    return h, rmsnorm_ref(h, w, eps)


def add_rmsnorm(x: torch.Tensor, r: torch.Tensor, w: torch.Tensor, eps: float = 1e-5):
    """``(h, y)`` with ``h = x + r`` (the new residual stream) and ``y = rmsnorm(h) * w``."""
    if x.is_cuda:
        return _AddRMSNorm.apply(x, r, w, eps)
    return add_rmsnorm_ref(x, r, w, eps)


# ------------------------------------------------------------------------------------ RoPE
def rope_tables(seq: int, head_dim: int, theta: float = 500000.0, device=None,
                scaling: dict | None = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 cos/sin tables [seq, head_dim/2] (Llama-3 RoPE; optional llama3 frequency scaling)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:  # Llama-3.1 style long-context scaling
        factor, lo, hi, orig = scaling["factor"], scaling["low_freq_factor"], scaling["high_freq_factor"], scaling["original_max_position_embeddings"]
        wavelen = 2 * torch.pi / inv
        smooth = ((orig / wavelen) - lo) / (hi - lo)
        scaled = torch.where(wavelen > orig / lo, inv / factor, inv)
        mid = (wavelen <= orig / lo) & (wavelen >= orig / hi)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(seq, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_split_ref(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, B: int, S: int, H: int, Hkv: int, Dh: int,
                   pos_offset: int = 0):
    x = qkv.view(B, S, H + 2 * Hkv, Dh).float()
    c = cos[pos_offset:pos_offset + S].view(1, S, 1, Dh // 2)
    s = sin[pos_offset:pos_offset + S].view(1, S, 1, Dh // 2)

    def rot(t):
        a, b = t[..., : Dh // 2], t[..., Dh // 2:]
        return torch.cat([a * c - b * s, b * c + a * s], dim=-1)

    q = rot(x[:, :, :H]).to(qkv.dtype).transpose(1, 2).contiguous()
    k = rot(x[:, :, H:H + Hkv]).to(qkv.dtype).transpose(1, 2).contiguous()
    v = x[:, :, H + Hkv:].to(qkv.dtype).transpose(1, 2).contiguous()
    return q, k, v


class _RopeSplit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, B, S, H, Hkv, Dh, pos_offset, want_t=False):
        q, k, v = hip().rope_split_fwd(qkv.contiguous(), cos, sin, B, S, H, Hkv, Dh, pos_offset)
        ctx.save_for_backward(cos, sin)
        ctx.meta = (pos_offset, qkv.shape)
        # backward also writes dqkv^T for the QKV weight gradient (rope_split_bwd_t, offered via offer_t)
        ctx.want_t = bool(want_t) and Dh == 128 and S % 64 == 0 and B * S // 64 <= 65535
        return q, k, v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        pos_offset, shape = ctx.meta
        if ctx.want_t:
            dqkv, dqkv_t = hip().rope_split_bwd_t(dq.contiguous(), dk.contiguous(), dv.contiguous(), cos, sin, pos_offset)
            out = dqkv.view(shape)
            offer_t(out, dqkv_t)
            return out, None, None, None, None, None, None, None, None, None
        dqkv = hip().rope_split_bwd(dq.contiguous(), dk.contiguous(), dv.contiguous(), cos, sin, pos_offset)
        return dqkv.view(shape), None, None, None, None, None, None, None, None, None


def rope_split(qkv, cos, sin, B, S, H, Hkv, Dh, pos_offset: int = 0, want_t: bool = False):
    """Fused QKV split + RoPE: [B*S, (H+2Hkv)*Dh] -> q [B,H,S,Dh], k/v [B,Hkv,S,Dh].  ``want_t``: the
    backward offers dqkv^T to the QKV projection's weight gradient (:func:`offer_t`)."""
    if qkv.is_cuda:
        return _RopeSplit.apply(qkv, cos, sin, B, S, H, Hkv, Dh, pos_offset, want_t)
    return rope_split_ref(qkv, cos, sin, B, S, H, Hkv, Dh, pos_offset)


# ------------------------------------------------------------------------------------ SwiGLU
def swiglu_ref(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (torch.nn.functional.silu(g) * u).to(gu.dtype)


def swiglu_bwd_ref(dh: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    """d[gate | up] of ``silu(g) * u`` (fp32 math, ``gu``'s dtype out)."""
    g, u = gu.float().chunk(2, dim=-1)
    d = dh.float()
    sg = torch.sigmoid(g)
    return torch.cat([d * u * sg * (1 + g * (1 - sg)), d * g * sg], dim=-1).to(gu.dtype)


def swiglu_bwd_t(dh: torch.Tensor, gu: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """SwiGLU backward returning ``(dgu [T, 2F], dgu^T [2F, T])``: the HIP kernel writes the transposed
    copy from its LDS tile (T, F multiples of 64); elsewhere the reference plus a transpose."""
    if gu.is_cuda and gu.dim() == 2 and gu.size(0) % 64 == 0 and (gu.size(1) // 2) % 128 == 0:
        # 64 x 128 tiles: 7 % faster than 64 x 64 at the Llama-3-8B shape (profiles/r04_llama)
        return tuple(hip().swiglu_bwd_t128(dh.contiguous(), gu.contiguous()))
    if gu.is_cuda and gu.dim() == 2 and gu.size(0) % 64 == 0 and (gu.size(1) // 2) % 64 == 0:
        dgu, dgu_t = hip().swiglu_bwd_t(dh.contiguous(), gu.contiguous())
        return dgu, dgu_t
    dgu = hip().swiglu_bwd(dh.contiguous(), gu.contiguous()) if gu.is_cuda else swiglu_bwd_ref(dh, gu)
    return dgu, transpose(dgu)


def swiglu_fwd_t(gu: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """SwiGLU forward returning ``(h [T, F], h^T [F, T])`` (no autograd): the HIP kernel writes the
    transposed copy from its LDS tile; elsewhere the reference plus a transpose."""
    if gu.is_cuda and gu.dim() == 2 and gu.size(0) % 64 == 0 and (gu.size(1) // 2) % 128 == 0:
        return tuple(hip().swiglu_fwd_t128(gu.contiguous()))
    if gu.is_cuda and gu.dim() == 2 and gu.size(0) % 64 == 0 and (gu.size(1) // 2) % 64 == 0:
        return tuple(hip().swiglu_fwd_t(gu.contiguous()))
    h = hip().swiglu_fwd(gu.contiguous()) if gu.is_cuda else swiglu_ref(gu)
    return h, transpose(h)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return hip().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dh):
        (gu,) = ctx.saved_tensors
        return hip().swiglu_bwd(dh.contiguous(), gu)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if gu.is_cuda:
        return _SwiGLU.apply(gu)
    return swiglu_ref(gu)


# ------------------------------------------------------------------------------------ loss
def cross_entropy_ref(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    return torch.nn.functional.cross_entropy(logits.float().view(-1, logits.size(-1)), labels.view(-1), ignore_index=ignore_index)


class _CrossEntropy(torch.autograd.Function):
    """Mean token cross-entropy; backward overwrites the (no longer needed) bf16 logits with dlogits.
    ``want_t``: the backward kernel also writes dlogits^T and offers it (:func:`offer_t`) to the lm_head
    weight gradient (xent_bwd_t, T multiple of 64, V of 128)."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index, want_t=False):
        V = logits.size(-1)
        lg = logits.contiguous().view(-1, V)
        lb = labels.contiguous().view(-1)
        loss_rows, lse = hip().xent_fwd(lg, lb, int(ignore_index))
        nvalid = (lb != ignore_index).sum().clamp_min(1).float()
        ctx.lg, ctx.lb, ctx.lse, ctx.nvalid, ctx.ii, ctx.shape = lg, lb, lse, nvalid, int(ignore_index), logits.shape
        ctx.want_t = bool(want_t) and lg.size(0) % 64 == 0 and V % 128 == 0 and lg.size(0) // 64 <= 65535
        return loss_rows.sum() / nvalid

    @staticmethod
    def backward(ctx, g):
        scale = (g.float() / ctx.nvalid).reshape(1).contiguous()
        lg = ctx.lg
        ctx.lg = None
        if ctx.want_t:
            lg_t = hip().xent_bwd_t(lg, ctx.lb, ctx.lse, scale, ctx.ii)
            out = lg.view(ctx.shape)
            offer_t(out, lg_t)
            return out, None, None, None
        hip().xent_bwd_inplace(lg, ctx.lb, ctx.lse, scale, ctx.ii)
        return lg.view(ctx.shape), None, None, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100, want_t: bool = False) -> torch.Tensor:
    if logits.is_cuda:
        return _CrossEntropy.apply(logits, labels, ignore_index, want_t)
    return cross_entropy_ref(logits, labels, ignore_index)


# ------------------------------------------------------------------------------------ attention
def attention_ref(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float | None = None) -> torch.Tensor:
    """fp32 causal GQA attention: q [B,H,S,D], k/v [B,Hkv,S,D] -> o [B,S,H,D] (same dtype as q)."""
    B, H, S, Dh = q.shape
    rep = H // k.size(1)
    kf = k.float().repeat_interleave(rep, dim=1)
    vf = v.float().repeat_interleave(rep, dim=1)
    sc = (scale if scale is not None else Dh ** -0.5)
    s = torch.matmul(q.float(), kf.transpose(-1, -2)) * sc
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    p = torch.softmax(s.masked_fill(mask, float("-inf")), dim=-1)
    return torch.matmul(p, vf).transpose(1, 2).to(q.dtype).contiguous()


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, with_t=False):
        ctx.set_materialize_grads(False)  # no zero-filled gradient for O^T (non-differentiable) in backward
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        if with_t:  # the kernel also writes O^T [H*D, B*S] (the o-projection's NT-layout x^T)
            o, lse, o_t = hip().attn_fwd_t(q, k, v, float(scale))
            ctx.mark_non_differentiable(o_t)
        else:
            o, lse = hip().attn_fwd(q, k, v, float(scale))
            o_t = None
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale = float(scale)
        return o, o_t

    @staticmethod
    def backward(ctx, do, _do_t=None):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = hip().attn_bwd(do.contiguous(), q, k, v, o, lse, ctx.scale)
        return dq, dk, dv, None, None


def flash_attention_supported(q: torch.Tensor, k: torch.Tensor) -> bool:
    return q.is_cuda and q.dtype == torch.bfloat16 and q.size(-1) == 128 and q.size(2) % 128 == 0 and q.size(1) % k.size(1) == 0


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float | None = None):
    """Causal GQA attention -> [B, S, H, D]; the HIP flash kernel on GPU (head dim 128, S % 128 == 0)."""
    sc = scale if scale is not None else q.size(-1) ** -0.5
    if q.is_cuda:
        if not flash_attention_supported(q, k):
            raise ValueError("HIP flash attention needs bf16, head dim 128 and S % 128 == 0")
        return _FlashAttention.apply(q, k, v, sc, False)[0]
    return attention_ref(q, k, v, sc)


def attention_t(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float | None = None):
    """``(o [B, S, H, D], o^T [H*D, B*S])``: on GPU the forward kernel writes the transposed copy from
    its LDS tile (no gradient flows through it); elsewhere the reference plus a transpose."""
    sc = scale if scale is not None else q.size(-1) ** -0.5
    if q.is_cuda:
        if not flash_attention_supported(q, k):
            raise ValueError("HIP flash attention needs bf16, head dim 128 and S % 128 == 0")
        return _FlashAttention.apply(q, k, v, sc, True)
    o = attention_ref(q, k, v, sc)
    B, S, H, D = o.shape
    return o, o.detach().reshape(B * S, H * D).t().contiguous()
