"""Flat-buffer AdamW with fp32 master weights (one fused HIP launch per step on MI355X).

State per parameter element: fp32 master, fp32 m, fp32 v (12 B) + the bf16 model weight and bf16
gradient that live in :class:`~.llama.FlatParams`.  The step reads 14 B and writes 14 B per element
— HBM-bound by construction, so it is one grid-stride kernel over the whole 8 B-element buffer
instead of one launch per tensor.  Hyper-parameters are a device tensor so nothing syncs the host.
Optional global-norm clipping uses one more fused pass (``sq_norm``) and stays on the device.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..ops import fused

__all__ = ["FlatAdamW"]


class FlatAdamW:
    def __init__(self, flat, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8, weight_decay: float = 0.1,
                 clip_norm: Optional[float] = 1.0):
        self.flat = flat
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.clip_norm = clip_norm
        self.master = flat.data.float()
        self.m = torch.zeros_like(self.master)
        self.v = torch.zeros_like(self.master)
        self.t = 0
        self.hp = torch.zeros(8, dtype=torch.float32, device=flat.data.device)

    def state_bytes(self) -> int:
        return 3 * self.master.numel() * 4

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0) -> None:
        self.t += 1
        b1, b2 = self.betas
        gs = torch.tensor(grad_scale, dtype=torch.float32, device=self.hp.device)
        if self.clip_norm is not None:
            if self.flat.grad.is_cuda:
                sq = fused.hip().sq_norm(self.flat.grad)
            else:
                sq = self.flat.grad.float().pow(2).sum()
            norm = sq.sqrt() * grad_scale
            gs = gs * torch.clamp(self.clip_norm / (norm + 1e-6), max=1.0)
        vals = torch.tensor([self.lr, b1, b2, self.eps, self.wd, 0.0, 1 - b1 ** self.t, 1 - b2 ** self.t], dtype=torch.float32)
        self.hp.copy_(vals, non_blocking=True)
        self.hp[5:6].copy_(gs.reshape(1))
        if self.flat.data.is_cuda:
            fused.hip().adamw_step(self.master, self.m, self.v, self.flat.grad, self.flat.data, self.hp)
        else:
            self._step_ref()

    def _step_ref(self) -> None:
        lr, b1, b2, eps, wd, gs, bc1, bc2 = self.hp.tolist()
        g = self.flat.grad.float() * gs
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        upd = (self.m / bc1) / ((self.v / bc2).sqrt() + eps)
        self.master.sub_(lr * (upd + wd * self.master))
        self.flat.data.copy_(self.master.to(self.flat.data.dtype))
