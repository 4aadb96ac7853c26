"""Flat-buffer AdamW with fp32 master weights (one fused HIP launch per step on MI355X).

State per parameter element: fp32 master, fp32 m, fp32 v (12 B) + the bf16 model weight and bf16
gradient that live in :class:`~.llama.FlatParams`.  The step reads 14 B and writes 14 B per element
— HBM-bound by construction, so it is one grid-stride kernel over the whole 8 B-element buffer
instead of one launch per tensor.  Hyper-parameters are a device tensor so nothing syncs the host.
Optional global-norm clipping uses one more fused pass (``sq_norm``) and stays on the device.

``shards`` (ZeRO-1, :class:`~..parallel.dp.BucketedAllReduce` with ``zero1=True``): the optimizer
owns only those flat-buffer ranges — its master/m/v hold their concatenation, one kernel launch per
range, and the clipping norm is the all-reduced sum of every rank's shard norms.

``capturable=True``: the step count and every hyper-parameter stay on the device (bias corrections
computed there), so a whole training step including :meth:`step` can be captured into a hipGraph and
replayed (``models/train.py --graph``); the host mirror ``t`` is advanced by :meth:`note_replay`.

Persistent transposed weights (``FlatParams.enable_transposed``, the NT-layout Llama): on a GPU without
shards the step is ``adamw_step_t`` -- the projection matrices by a 64 x 64-tile kernel that writes W
and W^T in the same pass, the rest of the buffer by the flat kernel -- and every W^T is valid after
it.  Any other path (ZeRO-1 shards, CPU) leaves W^T stale, and the backward re-makes it on first use.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops import fused

__all__ = ["FlatAdamW", "FlatSGD"]


class FlatAdamW:
    def __init__(self, flat, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8, weight_decay: float = 0.1,
                 clip_norm: Optional[float] = 1.0, shards: Optional[Sequence[Tuple[int, int]]] = None, group=None,
                 capturable: bool = False):
        self.flat = flat
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.clip_norm = clip_norm
        # AdamW-T tile kernel: how many 8-row passes' loads it issues before their stores (1, 2 or 4);
        # 2 measured fastest at the Llama-3-8B layout: 40.85 ms vs 42.51 (1) and 41.76 (4) (profiles/r04_memk)
        self.adamw_ahead = 2
        self.group = group
        self.sharded = shards is not None
        self.shards: List[Tuple[int, int]] = list(shards) if shards is not None else [(0, flat.numel)]
        if self.sharded:
            self.master = torch.cat([flat.data[s:e].float() for s, e in self.shards])
        else:
            self.master = flat.data.float()
        self.m = torch.zeros_like(self.master)
        self.v = torch.zeros_like(self.master)
        self.hp = torch.zeros(8, dtype=torch.float32, device=flat.data.device)
        self.capturable = capturable
        self.t_dev = torch.zeros(1, dtype=torch.float32, device=flat.data.device) if capturable else None
        self._t = 0
        self.hp_dev = None
        if capturable:
            b1, b2 = betas
            self.hp[:5].copy_(torch.tensor([lr, b1, b2, eps, weight_decay], dtype=torch.float32))
            # fused path (GPU, unsharded): [lr, b1, b2, eps, wd, grad_scale, clip_norm, -] for adamw_step_dev
            self.hp_dev = torch.tensor([lr, b1, b2, eps, weight_decay, 1.0, clip_norm if clip_norm else -1.0, 0.0],
                                       dtype=torch.float32).to(flat.data.device)
            self._hp_scale = 1.0
        self._deferred = []  # events the next step's writes must wait for (async checkpoint copies)
        # the fused W + W^T step (adamw_step_t) applies on a GPU without shards
        self.fused_t = (getattr(flat, "data_t", None) is not None and not self.sharded and flat.data.is_cuda)

    @property
    def t(self) -> int:
        """Optimizer steps taken (host view; checkpoints record it)."""
        return self._t

    @t.setter
    def t(self, value: int) -> None:
        self._t = int(value)
        if self.t_dev is not None:
            self.t_dev.fill_(float(self._t))

    def note_replay(self, n: int = 1) -> None:
        """A captured :meth:`step` ran ``n`` more times on the device: advance the host mirror."""
        self._t += n

    def defer_until(self, event) -> None:
        """Make the next :meth:`step` (on its stream) wait for ``event`` before it writes."""
        self._deferred.append(event)

    def state_bytes(self) -> int:
        return 3 * self.master.numel() * 4

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, sq: Optional[torch.Tensor] = None, grad: Optional[torch.Tensor] = None) -> None:
        """``sq``: this rank's precomputed sum of squared gradients over its shards (the
        data-parallel reducer's overlapped per-bucket norms); computed here when ``None``.
        ``grad``: the flat gradient to apply instead of the bf16 ``flat.grad`` -- the fp32 sum a DP
        reduction in fp32 leaves (``BucketedAllReduce.reduced_grad``); the kernels read either type."""
        gbuf = grad if grad is not None else self.flat.grad
        if self._deferred:
            cur = torch.cuda.current_stream(self.hp.device)
            for ev in self._deferred:
                cur.wait_event(ev)
            self._deferred.clear()
        if self.capturable:
            self._step_device(grad_scale, sq, gbuf)
            return
        self._t += 1
        b1, b2 = self.betas
        gs = torch.tensor(grad_scale, dtype=torch.float32, device=self.hp.device)
        if self.clip_norm is not None:
            for g in ([] if sq is not None else self._views(gbuf)):
                part = fused.hip().sq_norm(g) if g.is_cuda else g.float().pow(2).sum()
                sq = part if sq is None else sq + part
            if self.sharded and dist.is_initialized() and dist.get_world_size(self.group) > 1:
                dist.all_reduce(sq, group=self.group)
            norm = sq.sqrt() * grad_scale
            gs = gs * torch.clamp(self.clip_norm / (norm + 1e-6), max=1.0)
        vals = torch.tensor([self.lr, b1, b2, self.eps, self.wd, 0.0, 1 - b1 ** self.t, 1 - b2 ** self.t], dtype=torch.float32)
        self.hp.copy_(vals, non_blocking=True)
        self.hp[5:6].copy_(gs.reshape(1))
        if self.fused_t:
            mats, tiles, ranges, maxr = self.flat.adamw_plan()
            fused.hip().adamw_step_t(self.master, self.m, self.v, gbuf, self.flat.data, self.flat.data_t, self.hp,
                                     mats, tiles, ranges, maxr, None, None, self.adamw_ahead)
            self.flat.mark_t_valid()
            return
        self._invalidate_t()
        o = 0
        for (s, e), g, d in zip(self.shards, self._views(gbuf), self._views(self.flat.data)):
            n = e - s
            st = (self.master[o:o + n], self.m[o:o + n], self.v[o:o + n])
            if d.is_cuda:
                fused.hip().adamw_step(*st, g, d, self.hp)
            else:
                self._step_ref(*st, g, d)
            o += n

    def _clip_sq(self, sq: Optional[torch.Tensor], gbuf: torch.Tensor) -> torch.Tensor:
        for g in ([] if sq is not None else self._views(gbuf)):
            part = fused.hip().sq_norm(g) if g.is_cuda else g.float().pow(2).sum()
            sq = part if sq is None else sq + part
        if self.sharded and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(sq, group=self.group)
        return sq

    def _step_device(self, grad_scale: float, sq: Optional[torch.Tensor], gbuf: torch.Tensor) -> None:
        """Host-sync-free step: no host->device copies, so it captures.  On a GPU without shards it
        is two HIP launches — ``sq_norm_parts`` (clipping partials, step counter += 1) and
        ``adamw_step_dev`` (bias corrections and clip factor derived in-kernel)."""
        g, d = gbuf, self.flat.data
        if d.is_cuda and not self.sharded and sq is None:
            hip = fused.hip()
            if grad_scale != self._hp_scale:  # constant per run (1/world): set once, persists across replays
                self.hp_dev[5:6].fill_(grad_scale)
                self._hp_scale = grad_scale
            if self.clip_norm is not None:
                part = hip.sq_norm_parts(g, self.t_dev)
            else:
                part = None
                self.t_dev.add_(1.0)
            if not torch.cuda.is_current_stream_capturing():
                self._t += 1
            if self.fused_t:
                mats, tiles, ranges, maxr = self.flat.adamw_plan()
                hip.adamw_step_t(self.master, self.m, self.v, g, d, self.flat.data_t, self.hp_dev, mats, tiles, ranges, maxr,
                                 part, self.t_dev, 1)
                self.flat.mark_t_valid()
                return
            hip.adamw_step_dev(self.master, self.m, self.v, g, d, self.hp_dev, part, self.t_dev)
            self._invalidate_t()
            return
        b1, b2 = self.betas
        self.t_dev.add_(1.0)
        if not (self.t_dev.is_cuda and torch.cuda.is_current_stream_capturing()):
            self._t += 1
        self.hp[6:7].copy_(1.0 - torch.pow(b1, self.t_dev))
        self.hp[7:8].copy_(1.0 - torch.pow(b2, self.t_dev))
        if self.clip_norm is not None:
            norm = self._clip_sq(sq, gbuf).sqrt() * grad_scale
            self.hp[5:6].copy_((torch.clamp(self.clip_norm / (norm + 1e-6), max=1.0) * grad_scale).reshape(1))
        else:
            self.hp[5:6].fill_(grad_scale)
        self._invalidate_t()
        o = 0
        for (s, e), g, d in zip(self.shards, self._views(gbuf), self._views(self.flat.data)):
            n = e - s
            st = (self.master[o:o + n], self.m[o:o + n], self.v[o:o + n])
            if d.is_cuda:
                fused.hip().adamw_step(*st, g, d, self.hp)
            else:
                self._step_ref(*st, g, d)
            o += n

    def _invalidate_t(self) -> None:
        if hasattr(self.flat, "invalidate_t"):
            self.flat.invalidate_t()

    def _views(self, buf: torch.Tensor):
        return [buf[s:e] for s, e in self.shards]

    def _step_ref(self, master, m, v, grad, data) -> None:
        lr, b1, b2, eps, wd, gs, bc1, bc2 = self.hp.tolist()
        g = grad.float() * gs
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        upd = (m / bc1) / ((v / bc2).sqrt() + eps)
        master.sub_(lr * (upd + wd * master))
        data.copy_(master.to(data.dtype))


class FlatSGD:
    """Plain SGD on the flat buffer (fp32 master, no momentum, no weight decay, no clipping):
    ``w -= lr * grad_scale * g``.  The data-parallel parity check of ``models/train.py
    --optimizer sgd``: AdamW's update m / sqrt(v) is invariant to the scale of the
    gradient, so a k-rank run whose reduction never ran (each rank applying its local gradient / k)
    tracks the 1-rank run within tolerance; SGD's update is linear in the gradient, so it cannot.
    Same interface as :class:`FlatAdamW` (``shards`` for ZeRO-1, ``capturable`` for hipGraph steps,
    ``t_dev`` as the device step counter); not checkpointable."""

    _CHUNK = 1 << 26  # elements per fp32 temporary

    def __init__(self, flat, lr: float = 1e-2, shards: Optional[Sequence[Tuple[int, int]]] = None, group=None,
                 capturable: bool = False):
        self.flat = flat
        self.lr = float(lr)
        self.group = group
        self.sharded = shards is not None
        self.shards: List[Tuple[int, int]] = list(shards) if shards is not None else [(0, flat.numel)]
        if self.sharded:
            self.master = torch.cat([flat.data[s:e].float() for s, e in self.shards])
        else:
            self.master = flat.data.float()
        self.capturable = capturable
        self.t_dev = torch.zeros(1, dtype=torch.float32, device=flat.data.device) if capturable else None
        self._t = 0
        self._deferred = []
        self.fused_t = False

    @property
    def t(self) -> int:
        return self._t

    @t.setter
    def t(self, value: int) -> None:
        self._t = int(value)
        if self.t_dev is not None:
            self.t_dev.fill_(float(self._t))

    def note_replay(self, n: int = 1) -> None:
        self._t += n

    def defer_until(self, event) -> None:
        self._deferred.append(event)

    def state_bytes(self) -> int:
        return self.master.numel() * 4

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, sq: Optional[torch.Tensor] = None, grad: Optional[torch.Tensor] = None) -> None:
        gbuf = grad if grad is not None else self.flat.grad
        if self._deferred:
            cur = torch.cuda.current_stream(self.master.device)
            for ev in self._deferred:
                cur.wait_event(ev)
            self._deferred.clear()
        if self.t_dev is not None:
            self.t_dev.add_(1.0)
        if not (self.master.is_cuda and torch.cuda.is_current_stream_capturing()):
            self._t += 1
        alpha = -self.lr * float(grad_scale)
        o = 0
        for s, e in self.shards:
            for a in range(s, e, self._CHUNK):
                b = min(e, a + self._CHUNK)
                m = self.master[o + a - s:o + b - s]
                m.add_(gbuf[a:b].float(), alpha=alpha)
                self.flat.data[a:b].copy_(m)
            o += e - s
        if hasattr(self.flat, "invalidate_t"):
            self.flat.invalidate_t()
