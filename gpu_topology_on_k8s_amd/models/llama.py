"""Llama-3 decoder (random init) for the placement-validation workload (BASELINE config 5).

"Single pod requests 8 MI355X; Llama-3-8B DP all-reduce training on the allocated set, tokens/sec vs
worst-topology placement."  The reference has no model code; this is the workload
that turns a placement into a measurable training throughput.

MI355X-first layout:
  * every parameter is a view into ONE flat bf16 buffer and every gradient a view into ONE flat bf16
    gradient buffer (:class:`FlatParams`): the data-parallel engine all-reduces contiguous buckets of
    that buffer straight from the backward hooks, and the optimizer is one fused AdamW launch over
    the whole buffer (fp32 master + moments: 14 B/param read + 14 B/param written per step);
  * fused QKV and gate|up projections -> hipBLASLt GEMMs; everything between GEMMs is a fused HIP
    kernel (RMSNorm, RoPE + head split, SwiGLU, cross-entropy with in-place dlogits);
  * backward GEMMs in the forward GEMM's "NT" layout (``gemm_layout="nt"``): dgrad as
    ``dy (W^T)^T`` and wgrad as ``(dy^T)(x^T)^T`` -- hipBLASLt runs NT 10-40 % faster than the NN / TN
    layouts autograd would hand it (bench/gemm_layout_bench.py).  ``W^T`` stays resident and the
    optimizer rewrites it with ``W``; the transposed activations come from their producer kernels
    (SwiGLU ``h^T``, attention ``O^T``, RoPE-backward ``dqkv^T``, cross-entropy ``dlogits^T``) or from
    the LDS-tiled HIP transpose (``ops.fused.transpose``) for the rest.  Alternatives measured flat or
    slower on MI355X and retired in round 5 (records in profiles/ and docs/PERFORMANCE.md): transposes
    on a side stream in forward (r01), NN input gradients (r03_layout), x^T made in the forward and
    weight-gradient GEMMs on a side stream (r04_llama, r04_wgs), unfused residual adds (r01_fuse_res),
    autograd-accumulated norm / embedding gradients (r04_flatgrad);
  * Llama-3-8B = 8.03 B params: 16 GB bf16 weights + 16 GB bf16 grads + 96 GB fp32 master/m/v =
    128 GB, leaving ~160 GB of the 288 GB HBM for activations, so DP alone suffices (no TP/PP/SP).
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from ..ops import fused

__all__ = ["LlamaConfig", "FlatParams", "Llama", "smoke_step", "PROJECTIONS"]

#: the projections of a block (and the head), as named in the parameters
PROJECTIONS = ("wqkv", "wo", "w13", "w2", "lm_head")


@dataclass(frozen=True)
class LlamaConfig:
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    vocab: int = 128256
    ffn_dim: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq: int = 8192

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @classmethod
    def llama3_8b(cls) -> "LlamaConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "LlamaConfig":
        return cls(dim=256, n_layers=2, n_heads=4, n_kv_heads=2, vocab=1024, ffn_dim=512, max_seq=512)

    @classmethod
    def named(cls, name: str) -> "LlamaConfig":
        table = {
            "llama3-8b": cls.llama3_8b(),
            "tiny": cls.tiny(),
            "llama3-1b": cls(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, vocab=128256, ffn_dim=8192),
        }
        return table[name]

    def param_shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        D, Dh, H, Hkv = self.dim, self.head_dim, self.n_heads, self.n_kv_heads
        shapes: List[Tuple[str, Tuple[int, ...]]] = [("tok_emb", (self.vocab, D))]
        for i in range(self.n_layers):
            shapes += [
                (f"l{i}.attn_norm", (D,)),
                (f"l{i}.wqkv", ((H + 2 * Hkv) * Dh, D)),
                (f"l{i}.wo", (D, H * Dh)),
                (f"l{i}.ffn_norm", (D,)),
                (f"l{i}.w13", (2 * self.ffn_dim, D)),
                (f"l{i}.w2", (D, self.ffn_dim)),
            ]
        shapes += [("norm", (D,)), ("lm_head", (self.vocab, D))]
        return shapes

    def num_params(self) -> int:
        return sum(math.prod(s) for _, s in self.param_shapes())

    def flops_per_token(self, seq: int) -> float:
        """Training FLOPs per token: 6 N (dense) + 12 L S D (causal attention fwd+bwd, halved for causality)."""
        return 6.0 * self.num_params() + 6.0 * self.n_layers * seq * self.dim

    def to_dict(self) -> Dict[str, object]:
        return asdict(self)


_ALIGN = 64  # elements: keeps every parameter view 128-B aligned for 16-B vector kernels


class _ReadyHandle:
    def __init__(self, hooks: List[Callable], fn: Callable):
        self._hooks, self._fn = hooks, fn

    def remove(self) -> None:
        if self._fn in self._hooks:
            self._hooks.remove(self._fn)


class FlatParams:
    """All parameters as views of one flat bf16 buffer, gradients as views of one flat grad buffer.

    Projection weights can be marked *direct* (:class:`_FlatLinear`): their weight-gradient GEMM
    writes ``dW = dY^T X`` straight into the flat gradient view (``torch.mm(out=)``, ``addmm_`` when
    accumulating) instead of allocating a temporary that AccumulateGrad then adds in — no add
    kernel, no 16 GB zero-fill per step.  Readiness of a direct gradient is announced through
    :meth:`add_ready_hook` (the data-parallel bucket countdown), since no AccumulateGrad runs.
    """

    def __init__(self, shapes: List[Tuple[str, Tuple[int, ...]]], device, dtype=torch.bfloat16):
        self.names = [n for n, _ in shapes]
        self.shapes = {n: s for n, s in shapes}
        self.offsets: Dict[str, int] = {}
        off = 0
        for n, s in shapes:
            self.offsets[n] = off
            off += (math.prod(s) + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = off
        self.data = torch.zeros(off, dtype=dtype, device=device)
        self.grad = torch.zeros(off, dtype=dtype, device=device)
        self.params: Dict[str, torch.nn.Parameter] = {}
        for n, s in shapes:
            o, k = self.offsets[n], math.prod(s)
            p = torch.nn.Parameter(self.data[o:o + k].view(s))
            p.grad = self.grad[o:o + k].view(s)
            self.params[n] = p
        self.direct: Dict[str, bool] = {}  # name -> "fresh" (not yet written since zero_grad)
        self._ready: Dict[str, List[Callable]] = {}
        # persistent transposed weights (enable_transposed): W^T of each listed matrix in one flat
        # bf16 buffer, written by the optimizer's fused step or re-made lazily when stale
        self.data_t: Optional[torch.Tensor] = None
        self.t_offsets: Dict[str, int] = {}
        self.t_valid: Dict[str, bool] = {}
        self._t_ver: Dict[str, int] = {}  # data._version when each W^T was last made valid
        self.t_refreshes = 0  # lazy W^T re-makes (transposes) since construction
        self._plan = None  # adamw_plan() cache
        # NT layout: producers that hold a tile in LDS write the transposed copy too (SwiGLU h^T,
        # attention O^T, RoPE-backward dqkv^T, cross-entropy dlogits^T)
        self.producer_xt = False

    # ---------------------------------------------------------------- persistent W^T
    def enable_transposed(self, names) -> List[str]:
        """Keep ``W^T`` of the listed 2-D parameters resident: the NT-layout input
        gradient reads it every backward, and W changes only in the optimizer, which writes W^T in the
        same pass (``FlatAdamW`` + ``adamw_step_t``).  Matrices whose dims are not multiples of the fused
        tile kernel's 64 x 256 tile are left out.  -> the names kept."""
        want = set(names)
        keep = [n for n in self.names if n in want and len(self.shapes[n]) == 2
                and self.shapes[n][0] % 64 == 0 and self.shapes[n][1] % 256 == 0]
        off = 0
        self.t_offsets = {}
        for n in keep:
            self.t_offsets[n] = off
            off += (math.prod(self.shapes[n]) + _ALIGN - 1) // _ALIGN * _ALIGN
        self.data_t = torch.empty(off, dtype=self.data.dtype, device=self.data.device) if keep else None
        self.t_valid = {n: False for n in keep}
        self._plan = None
        return keep

    def weight_t(self, name: str) -> Optional[torch.Tensor]:
        """``W^T`` ([in, out], contiguous) of a transposed parameter, re-made first if stale; ``None``
        when ``name`` keeps no transposed copy."""
        if name not in self.t_offsets:
            return None
        R, C = self.shapes[name]
        o = self.t_offsets[name]
        view = self.data_t[o:o + R * C].view(C, R)
        # stale if invalidated, or if torch wrote the weights in place since (copy_, add_ ... bump the
        # flat buffer's version counter; kernels and collectives do not, so their callers invalidate)
        if not self.t_valid[name] or self._t_ver.get(name) != self.data._version:
            w = self.params[name].detach()
            if view.is_cuda:
                fused.hip().transpose_bf16_out(w.contiguous(), view)
            else:
                view.copy_(w.t())
            self.t_valid[name] = True
            self._t_ver[name] = self.data._version
            self.t_refreshes += 1
        return view

    def invalidate_t(self) -> None:
        """The weights changed outside the optimizer's fused step (init, broadcast, ZeRO-1 all-gather,
        checkpoint restore, an unfused optimizer): every W^T is re-made at its next use."""
        for n in self.t_valid:
            self.t_valid[n] = False

    def mark_t_valid(self) -> None:
        """The optimizer's fused step just wrote every W^T from the new W."""
        ver = self.data._version
        for n in self.t_valid:
            self.t_valid[n] = True
            self._t_ver[n] = ver

    def adamw_plan(self):
        """Descriptors of ``adamw_step_t``: (mats int64 [N, 5] = (offset, W^T offset, R, C, first tile),
        total 64x256 tiles, ranges int64 [M, 2] = the rest of the flat buffer as (start, length), longest
        range), on the buffer's device.  Cached."""
        if self._plan is None:
            mats, base, spans = [], 0, []
            for n in self.names:
                if n in self.t_offsets:
                    R, C = self.shapes[n]
                    mats.append((self.offsets[n], self.t_offsets[n], R, C, base))
                    base += (R // 64) * (C // 256)
                    spans.append((self.offsets[n], self.offsets[n] + R * C))
            ranges, cur = [], 0
            for a, b in sorted(spans):
                if a > cur:
                    ranges.append((cur, a - cur))
                cur = b
            if cur < self.numel:
                ranges.append((cur, self.numel - cur))
            dev = self.data.device
            mt = torch.tensor(mats or [[0] * 5], dtype=torch.int64)[: len(mats)].to(dev)
            rt = torch.tensor(ranges or [[0, 0]], dtype=torch.int64)[: len(ranges)].to(dev)
            self._plan = (mt, base, rt, max((ln for _, ln in ranges), default=0))
        return self._plan

    def mark_direct(self, name: str) -> None:
        self.direct[name] = True

    def add_ready_hook(self, name: str, fn: Callable) -> _ReadyHandle:
        hooks = self._ready.setdefault(name, [])
        hooks.append(fn)
        return _ReadyHandle(hooks, fn)

    def write_grad(self, name: str, dy: torch.Tensor, x: Optional[torch.Tensor], nt: bool = False,
                   dy_t: Optional[torch.Tensor] = None, x_t: Optional[torch.Tensor] = None) -> None:
        """Weight gradient of ``y = x W^T`` into the flat buffer: ``W.grad (+)= dy^T x``.

        ``nt``: compute it as ``(dy^T)(x^T)^T`` from transposed copies, the GEMM layout hipBLASLt runs
        fastest (both operands contiguous along the token dimension being reduced); ``dy_t`` / ``x_t``
        are transposed copies their producer kernels wrote (SwiGLU backward, cross-entropy, RoPE)."""
        view = self.params[name].grad
        if nt:
            a = dy_t if dy_t is not None else fused.transpose(dy)
            b = (x_t if x_t is not None else fused.transpose(x)).t()
        else:
            a, b = dy.t(), x
        if self.direct[name]:
            torch.mm(a, b, out=view)
            self.direct[name] = False
        else:
            view.addmm_(a, b)
        for fn in list(self._ready.get(name, ())):
            fn(self.params[name])

    def grad_target(self, name: str) -> Tuple[torch.Tensor, bool]:
        """Where a kernel that writes ``name``'s whole gradient (norm / embedding backward) should write:
        ``(view, True)`` -- the flat slot itself -- on the first write since :meth:`zero_grad`; after
        that ``(scratch, False)``: the caller writes a scratch tensor and :meth:`mark_written` adds it
        in, so a second backward before ``zero_grad`` accumulates as autograd would."""
        view = self.params[name].grad
        if self.direct.get(name, False):
            return view, True
        return torch.empty_like(view), False

    def mark_written(self, name: str, partial: Optional[torch.Tensor] = None) -> None:
        """A kernel wrote ``name``'s gradient into the flat buffer itself (not through
        :meth:`write_grad`), or into ``partial`` (a :meth:`grad_target` scratch, added in here): clear
        its fresh flag and announce readiness (data-parallel buckets)."""
        if partial is not None:
            self.params[name].grad.add_(partial)
        self.direct[name] = False
        for fn in list(self._ready.get(name, ())):
            fn(self.params[name])

    def fill_unwritten(self) -> None:
        """Zero the gradients of direct parameters that received none since :meth:`zero_grad`."""
        for n, fresh in self.direct.items():
            if fresh:
                o, e = self.span(n)
                self.grad[o:e].zero_()

    def attach_grads(self) -> None:
        """(Re)bind every ``param.grad`` to its view of the flat gradient buffer."""
        for n, p in self.params.items():
            o, k = self.offsets[n], math.prod(self.shapes[n])
            p.grad = self.grad[o:o + k].view(self.shapes[n])

    def zero_grad(self) -> None:
        if not self.direct:
            self.grad.zero_()
            return
        for o, e in self._zero_runs():  # direct gradients are overwritten by their first writer instead
            self.grad[o:e].zero_()
        for n in self.direct:
            self.direct[n] = True

    def _zero_runs(self) -> List[Tuple[int, int]]:
        """Maximal runs of consecutive non-direct parameters (alignment padding included): one fill
        kernel per run instead of one per parameter."""
        key = tuple(sorted(self.direct))
        if getattr(self, "_runs_key", None) != key:
            runs: List[Tuple[int, int]] = []
            for n in self.names:
                o = self.offsets[n]
                e = self.span(n)[1]
                if n in self.direct:
                    continue
                if runs and runs[-1][1] >= o - (_ALIGN - 1) and self._only_padding(runs[-1][1], o):
                    runs[-1] = (runs[-1][0], e)
                else:
                    runs.append((o, e))
            self._runs, self._runs_key = runs, key
        return self._runs

    def _only_padding(self, a: int, b: int) -> bool:
        """True when no parameter starts in [a, b) (the gap is alignment padding, zero anyway)."""
        return all(not (a <= self.offsets[n] < b) for n in self.names)

    def span(self, name: str) -> Tuple[int, int]:
        o = self.offsets[name]
        return o, o + math.prod(self.shapes[name])


class _NTOperands:
    """``x^T`` and ``W^T`` of one forward GEMM for its NT-layout backward GEMMs: ``x^T`` as its producer
    kernel wrote it (``x_t``), else made from the kept ``x`` in backward by the HIP transpose; ``W^T``
    the persistent copy (``wt_fn``, :meth:`FlatParams.weight_t`), else transposed in backward."""

    def __init__(self, x: torch.Tensor, w: torch.Tensor, wt_fn: Optional[Callable[[], Optional[torch.Tensor]]] = None,
                 x_t: Optional[torch.Tensor] = None):
        self.wt_fn = wt_fn
        self.x_t = x_t
        self.x = None if x_t is not None else x
        self.w = w

    def get(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """-> (x^T, W^T), ready for use on the current stream."""
        x_t = self.x_t if self.x_t is not None else fused.transpose(self.x)
        w_t = self.wt_fn() if self.wt_fn is not None else None
        if w_t is None:
            w_t = fused.transpose(self.w)
        self.x = self.w = self.x_t = None
        return x_t, w_t


def _wt_fn(flat: "FlatParams", name: str):
    return (lambda: flat.weight_t(name)) if name in flat.t_offsets else None


class _FlatLinear(torch.autograd.Function):
    """``y = x W^T`` whose weight gradient is written in place into the flat buffer."""

    @staticmethod
    def forward(ctx, x, w, flat, name, nt, x_t=None):
        ctx.flat, ctx.name, ctx.nt = flat, name, nt
        if nt:
            ctx.ops = _NTOperands(x, w, _wt_fn(flat, name), x_t=x_t)
        else:
            ctx.save_for_backward(x)
            ctx.w = w  # a flat-buffer view: not version-checked (see _FlatRMSNorm)
        return F.linear(x, w)

    @staticmethod
    def backward(ctx, dy):
        if ctx.nt:
            x_t, w_t = ctx.ops.get()
            ctx.ops = None
            dy_t = fused.take_t(dy)  # dy^T written by dy's producer kernel (xent / RoPE backward), if any
            dx = F.linear(dy, w_t) if ctx.needs_input_grad[0] else None  # dy (W^T)^T
            ctx.flat.write_grad(ctx.name, dy, None, nt=True, x_t=x_t, dy_t=dy_t)
        else:
            (x,), w = ctx.saved_tensors, ctx.w
            ctx.w = None
            dx = dy.mm(w) if ctx.needs_input_grad[0] else None
            ctx.flat.write_grad(ctx.name, dy, x)
        return dx, None, None, None, None, None


class _FlatLinearSwiGLU(torch.autograd.Function):
    """``silu(g) * u`` of ``[g | u] = x W13^T``: the gate|up projection and SwiGLU as one node, so the
    backward gets d[g | u] AND its transpose from one HIP kernel (``fused.swiglu_bwd_t``) and feeds
    the transpose straight to the NT weight-gradient GEMM; the forward kernel writes ``h^T`` for the
    down projection's weight gradient."""

    @staticmethod
    def forward(ctx, x, w, flat, name, nt):
        ctx.set_materialize_grads(False)  # no zero-filled gradient for a^T (non-differentiable) in backward
        gu = F.linear(x, w)
        ctx.flat, ctx.name, ctx.nt = flat, name, nt
        if nt:
            ctx.ops = _NTOperands(x, w, _wt_fn(flat, name))
            ctx.save_for_backward(gu)
        else:
            ctx.save_for_backward(gu, x)
            ctx.w = w
        a_t = None
        if not gu.is_cuda:
            a = fused.swiglu_ref(gu)
        elif nt and flat.producer_xt and gu.size(0) % 64 == 0 and (gu.size(1) // 2) % 64 == 0:
            a, a_t = fused.swiglu_fwd_t(gu)  # the next projection's x^T from the same kernel
            ctx.mark_non_differentiable(a_t)
        else:
            a = fused.hip().swiglu_fwd(gu)
        return a, a_t

    @staticmethod
    def backward(ctx, da, _da_t=None):
        gu = ctx.saved_tensors[0]
        if ctx.nt:
            dgu, dgu_t = fused.swiglu_bwd_t(da, gu)
            x_t, w_t = ctx.ops.get()
            ctx.ops = None
            dx = F.linear(dgu, w_t) if ctx.needs_input_grad[0] else None
            ctx.flat.write_grad(ctx.name, dgu, None, nt=True, dy_t=dgu_t, x_t=x_t)
        else:
            (_, x), w = ctx.saved_tensors, ctx.w
            ctx.w = None
            dgu = fused.hip().swiglu_bwd(da.contiguous(), gu) if gu.is_cuda else fused.swiglu_bwd_ref(da, gu)
            dx = dgu.mm(w) if ctx.needs_input_grad[0] else None
            ctx.flat.write_grad(ctx.name, dgu, x)
        return dx, None, None, None, None


class _FlatRMSNorm(torch.autograd.Function):
    """``rmsnorm(x) * w`` whose weight gradient the backward kernel writes straight into the weight's
    slot of the flat gradient buffer (``rmsnorm_bwd_into``): no separate dW for autograd to add in,
    and no zero-fill of that slot in ``zero_grad`` (the weight is a direct parameter).

    The weight is kept on ``ctx``, not saved for backward: every parameter is a view of the flat
    buffer and views share one version counter, so ZeRO-1's all-gather of ANOTHER bucket landing
    during the forward (overlapped, parallel/dp.py ``gather_params``) would fail autograd's check
    although this weight's own bucket was gathered before its first use (``wait_param``) and nothing
    writes it again before the backward."""

    @staticmethod
    def forward(ctx, x, w, flat, name, eps):
        x = x.contiguous()
        y, rstd = fused.hip().rmsnorm_fwd(x, w, float(eps))
        ctx.save_for_backward(x, rstd)
        ctx.w, ctx.flat, ctx.name = w, flat, name
        return y

    @staticmethod
    def backward(ctx, dy):
        (x, rstd), w = ctx.saved_tensors, ctx.w
        ctx.w = None
        out, fresh = ctx.flat.grad_target(ctx.name)
        dx = fused.hip().rmsnorm_bwd_into(dy.contiguous(), x, w, rstd, out)
        ctx.flat.mark_written(ctx.name, None if fresh else out)
        return dx, None, None, None, None


class _FlatAddRMSNorm(torch.autograd.Function):
    """``h = x + r; y = rmsnorm(h) * w`` (ops/fused.py ``add_rmsnorm``) with the weight gradient written
    into the flat buffer by the backward kernel, as :class:`_FlatRMSNorm`."""

    @staticmethod
    def forward(ctx, x, r, w, flat, name, eps):
        h, y, rstd = fused.hip().add_rmsnorm_fwd(x.contiguous(), r.contiguous(), w, float(eps))
        ctx.save_for_backward(h, rstd)
        ctx.w, ctx.flat, ctx.name = w, flat, name  # not version-checked: see _FlatRMSNorm
        return h, y

    @staticmethod
    def backward(ctx, dh, dy):
        (h, rstd), w = ctx.saved_tensors, ctx.w
        ctx.w = None
        if dy is None:
            dy = torch.zeros_like(h)
        out, fresh = ctx.flat.grad_target(ctx.name)
        if dh is None:
            dx = fused.hip().rmsnorm_bwd_into(dy.contiguous(), h, w, rstd, out)
        else:
            dx = fused.hip().add_rmsnorm_bwd_into(dy.contiguous(), h, w, rstd, dh.contiguous(), out)
        ctx.flat.mark_written(ctx.name, None if fresh else out)
        return dx, dx, None, None, None, None


class _FlatEmbedding(torch.autograd.Function):
    """Token embedding whose gradient goes straight into the flat buffer: the slot is zeroed and
    ``embed_bwd_into`` sums each token's dx rows in position order (deterministic) -- instead of
    torch's embedding backward building a dense [V, D] gradient that autograd then adds in.  ``w`` is
    the Parameter itself (the only differentiable input); its autograd gradient is None."""

    @staticmethod
    def forward(ctx, tokens, w, flat, name):
        ctx.save_for_backward(tokens)
        ctx.flat, ctx.name = flat, name
        return F.embedding(tokens, w.detach())

    @staticmethod
    def backward(ctx, dy):
        (tokens,) = ctx.saved_tensors
        out, fresh = ctx.flat.grad_target(ctx.name)
        srt, perm = torch.sort(tokens.reshape(-1), stable=True)
        out.zero_()
        fused.hip().embed_bwd_into(srt, perm, dy.contiguous().view(-1, out.size(1)), out)
        ctx.flat.mark_written(ctx.name, None if fresh else out)
        return None, None, None, None


class Llama(torch.nn.Module):
    def __init__(self, cfg: LlamaConfig, device="cuda", seed: int = 0, checkpoint: bool = False, attn: str = "hip",
                 gemm_layout: str = "nt", persistent_wt: bool = True):
        """``gemm_layout``: "nt" (the GPU default, see the module docstring) or "native" (autograd's
        layouts: the reference the NT path is checked against).  ``persistent_wt=False`` re-makes every
        W^T by a transpose in every backward (the round-3 path; A/B reference for the AdamW-written W^T)."""
        super().__init__()
        if gemm_layout not in ("nt", "native"):
            raise ValueError("gemm_layout must be 'nt' or 'native'")
        self.cfg = cfg
        self.checkpoint = checkpoint
        self.attn = attn
        self.gemm_layout = gemm_layout
        # called with a parameter name before its first use in forward (ZeRO-1: wait for that
        # bucket's weight all-gather, parallel/dp.py BucketedAllReduce.wait_param)
        self.param_ready: Optional[Callable[[str], None]] = None
        self.flat = FlatParams(cfg.param_shapes(), device)
        # on the GPU every gradient is written straight into the flat buffer by its kernel (projections:
        # the weight-gradient GEMM; norms and the embedding: their backward kernels), so no parameter is
        # zero-filled and then accumulated into; on the CPU reference path norms and the embedding go
        # through autograd's accumulation
        self.flat_grads = torch.device(device).type == "cuda"
        for n, p in self.flat.params.items():
            self.register_parameter(n.replace(".", "_"), p)
            if (p.dim() == 2 and n != "tok_emb") or self.flat_grads:
                self.flat.mark_direct(n)
        self._init(seed)
        # NT layout: the producers that hold a tile in LDS write the transposed activation too, the
        # attention forward's epilogue O^T among them; W^T of every projection stays resident and the
        # optimizer rewrites it with W (no per-step weight transposes)
        self.flat.producer_xt = gemm_layout == "nt"
        self.attn_ot = self.flat.producer_xt
        self.persistent_wt = persistent_wt and gemm_layout == "nt"
        if self.persistent_wt:
            self.flat.enable_transposed([n for n in self.flat.direct if n != "tok_emb"])
        cos, sin = fused.rope_tables(cfg.max_seq, cfg.head_dim, cfg.rope_theta, device=device)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)

    @torch.no_grad()
    def _init(self, seed: int) -> None:
        self.flat.invalidate_t()
        dev = self.flat.data.device
        g = torch.Generator(device=dev).manual_seed(seed)  # same seed + device type => identical replicas
        std = 0.02
        out_std = std / math.sqrt(2 * self.cfg.n_layers)
        for n, p in self.flat.params.items():
            if n.endswith("norm"):
                p.fill_(1.0)
                continue
            s = out_std if (n.endswith(".wo") or n.endswith(".w2")) else std
            flat = p.view(-1)
            step = 1 << 26  # bounded fp32 scratch (256 MB) per chunk
            for i in range(0, flat.numel(), step):
                m = min(step, flat.numel() - i)
                flat[i:i + m].copy_(torch.randn(m, generator=g, dtype=torch.float32, device=dev).mul_(s))

    def P(self, name: str) -> torch.nn.Parameter:
        if self.param_ready is not None:
            self.param_ready(name)
        return self.flat.params[name]

    def _linear(self, x: torch.Tensor, name: str, x_t: Optional[torch.Tensor] = None) -> torch.Tensor:
        return _FlatLinear.apply(x, self.P(name).detach(), self.flat, name, self.gemm_layout == "nt", x_t)

    # ---------------------------------------------------------------- blocks
    def _attention(self, q, k, v, want_t: bool = False):
        """q [B,H,S,Dh], k/v [B,Hkv,S,Dh] -> [B,S,H,Dh] (token-major, what the o-projection reads);
        ``want_t``: ``(o, o^T [H*Dh, B*S])`` with the transposed copy written by the forward kernel."""
        if self.attn == "hip" and (not q.is_cuda or fused.flash_attention_supported(q, k)):
            if want_t:
                return fused.attention_t(q, k, v)
            return fused.attention(q, k, v)  # HIP MFMA flash attention (PyTorch reference on CPU)
        if self.attn in ("hip", "sdpa"):  # library SDPA: A/B baseline, or shapes the HIP kernel does not cover
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=q.size(1) != k.size(1))
        else:  # "sdpa-expand": explicit GQA expansion for SDPA backends without native GQA
            rep = q.size(1) // k.size(1)
            if rep > 1:
                k = k.repeat_interleave(rep, dim=1)
                v = v.repeat_interleave(rep, dim=1)
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        o = o.transpose(1, 2)
        return (o, None) if want_t else o

    def _norm(self, x: torch.Tensor, r: Optional[torch.Tensor], name: str):
        """``(x + r, rmsnorm(x + r))`` — the residual add fused into the norm kernel; ``r=None``
        is a plain norm of ``x`` (first layer)."""
        if self.flat_grads:
            w = self.P(name).detach()
            if r is None:
                return x, _FlatRMSNorm.apply(x, w, self.flat, name, self.cfg.norm_eps)
            return _FlatAddRMSNorm.apply(x, r, w, self.flat, name, self.cfg.norm_eps)
        if r is None:
            return x, fused.rmsnorm(x, self.P(name), self.cfg.norm_eps)
        return fused.add_rmsnorm(x, r, self.P(name), self.cfg.norm_eps)

    def _layer(self, i: int, x: torch.Tensor, B: int, S: int, r: Optional[torch.Tensor] = None):
        """One block; returns ``(x, r)``: the residual stream and the block's last branch output, which
        the next block's (or the final) norm adds in its own kernel."""
        cfg = self.cfg
        H, Hkv, Dh = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        x, h = self._norm(x, r, f"l{i}.attn_norm")
        qkv = self._linear(h, f"l{i}.wqkv")
        q, k, v = fused.rope_split(qkv, self.rope_cos, self.rope_sin, B, S, H, Hkv, Dh, want_t=self.flat.producer_xt)
        if self.attn_ot:
            # o^T from the attention kernel's epilogue: +47 us per layer in the kernel against the 43 us
            # transpose it replaces, step time unchanged in an interleaved A/B, +4.3 GB kept from the
            # forward (profiles/r04_otab)
            o, o_t = self._attention(q, k, v, want_t=True)
        else:
            o, o_t = self._attention(q, k, v), None
        o = o.reshape(B * S, H * Dh)  # [B, S, H, Dh] -> [B*S, H*Dh]
        x, h = self._norm(x, self._linear(o, f"l{i}.wo", x_t=o_t), f"l{i}.ffn_norm")
        a, a_t = _FlatLinearSwiGLU.apply(h, self.P(f"l{i}.w13").detach(), self.flat, f"l{i}.w13", self.gemm_layout == "nt")
        return x, self._linear(a, f"l{i}.w2", x_t=a_t)

    def forward(self, tokens: torch.Tensor, labels: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, S = tokens.shape
        fused.clear_t()  # transposed gradients a previous backward offered and nobody took
        if self.flat_grads:
            x = _FlatEmbedding.apply(tokens.reshape(-1), self.P("tok_emb"), self.flat, "tok_emb")  # [B*S, D]
        else:
            x = F.embedding(tokens.reshape(-1), self.P("tok_emb"))  # [B*S, D]
        r = None
        for i in range(self.cfg.n_layers):
            if self.checkpoint and self.training:
                x, r = torch.utils.checkpoint.checkpoint(self._layer, i, x, B, S, r, use_reentrant=False)
            else:
                x, r = self._layer(i, x, B, S, r)
        _, x = self._norm(x, r, "norm")
        logits = self._linear(x, "lm_head")  # [B*S, V]
        if labels is None:
            return logits.view(B, S, -1)
        return fused.cross_entropy(logits, labels.reshape(-1), want_t=self.flat.producer_xt)


def smoke_step(device: str = "cuda:0") -> float:
    """One tiny forward+backward on ``device`` through the HIP kernels (``__graft_entry__.smoke``): head
    dim 128 and multiples of the tile sizes, so the flash attention (with its O^T epilogue), the
    transposed-output SwiGLU / RoPE / cross-entropy kernels and the flat-gradient norm and embedding
    kernels all run, not their fallbacks."""
    torch.manual_seed(0)
    cfg = LlamaConfig(dim=512, n_layers=2, n_heads=4, n_kv_heads=2, vocab=1024, ffn_dim=1024, max_seq=512)
    model = Llama(cfg, device=device)
    tokens = torch.randint(0, cfg.vocab, (2, 128), device=device)
    assert model.attn_ot and model.flat_grads and model.persistent_wt
    loss = model(tokens, torch.roll(tokens, -1, dims=1))
    loss.backward()
    torch.cuda.synchronize()
    assert not fused._PENDING_T  # every transposed gradient a producer offered was consumed
    g = model.flat.grad.float()
    assert torch.isfinite(g).all() and g.abs().sum() > 0
    return float(loss.item())
