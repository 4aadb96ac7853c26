"""MNIST CNN — the workload of the Gaia paper's end-to-end experiment (Exp. 6).

Reference: the paper trains "the official MNIST sample" on Caffe, PyTorch and TensorFlow, once on the
GPU pair default Kubernetes picks and once on the pair Gaia picks, and compares mean training time
over 10 runs (paper p.7 Figs. 11-12; SURVEY.md §4 "End-to-end workload", §6 rows "MNIST training
time").  The architecture is the PyTorch example's: conv 1->32 3x3, conv 32->64 3x3, 2x2 max-pool,
dropout 0.25, fc 9216->128, dropout 0.5, fc 128->10 (1.2 M parameters).

MI355X-first: at the example's batch of 64 a step is ~100 kernels of a few µs each through the
library path (MIOpen convolutions with their layout transposes, casts and bias reductions), so it is
bound by launch latency, not by MFMA throughput or HBM.  The design therefore minimises launches:

* parameters and gradients are views of ONE flat bf16 buffer (:class:`~.llama.FlatParams`), so the
  data-parallel gradient reduction is one 2.4 MB RCCL all-reduce and AdamW one fused HIP launch
  (:class:`~.optim.FlatAdamW`);
* batches are synthesised on the device (no host->device copy per step);
* the whole step — batch synthesis, forward, backward, gradient all-reduce, clipping, AdamW — is
  captured once into a hipGraph and replayed (``models/train.py --graph``), one host launch per step;
* the classifier head is two library GEMMs per direction around four HIP kernels (ReLU+dropout and
  softmax cross-entropy, forward and backward, each also producing a bias gradient), with the
  weight-gradient GEMMs writing the flat buffer (no zero fills, no AccumulateGrad adds);
* the convolution stack is five hand-written HIP launches (``csrc/ops/mnist_conv.hip``): conv1+ReLU;
  conv2+ReLU+2x2 max-pool+dropout as one MFMA implicit GEMM whose accumulator rows are the pooling
  windows; backward as an MFMA dgrad that rebuilds dy2 from the pooled gradient and folds conv1's
  weight gradient into its epilogue, an MFMA wgrad, and a deterministic partial-sum reduction that
  writes the flat gradient directly.  ``conv="torch"`` keeps the library path for A/B and CPU.

Parameter layouts are channels-last: ``conv1.w`` [32,3,3,1], ``conv2.w`` [64,3,3,32] (co, ky, kx,
ci) and fc1 reads the pooled map in NHWC order — the same function class as the PyTorch example
(a fixed permutation of its parameters).

Data is synthetic and MNIST-shaped (no dataset download: no network): ten fixed 28x28 class
prototypes (seeded, identical on every rank) plus Gaussian noise, normalised with MNIST's mean/std;
the label is the prototype's class, so the loss falls the way it does on real digits.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import torch
import torch.nn.functional as F

from .llama import FlatParams

__all__ = ["MnistConfig", "MnistCNN", "EPOCH_IMAGES"]

EPOCH_IMAGES = 60000  # MNIST training split
_MEAN, _STD = 0.1307, 0.3081


@dataclass(frozen=True)
class MnistConfig:
    c1: int = 32
    c2: int = 64
    hidden: int = 128
    classes: int = 10
    image: int = 28
    p1: float = 0.25
    p2: float = 0.5
    noise: float = 0.6  # per-pixel noise std on the [0, 1] prototype images

    @staticmethod
    def named(name: str) -> "MnistConfig":
        if name == "mnist-cnn":
            return MnistConfig()
        raise ValueError(f"unknown MNIST model {name!r}")

    @property
    def pooled(self) -> int:
        return self.c2 * ((self.image - 4) // 2) ** 2  # two valid 3x3 convs, one 2x2 pool

    def param_shapes(self):
        return [("conv1.w", (self.c1, 3, 3, 1)), ("conv1.b", (self.c1,)),
                ("conv2.w", (self.c2, 3, 3, self.c1)), ("conv2.b", (self.c2,)),
                ("fc1.w", (self.hidden, self.pooled)), ("fc1.b", (self.hidden,)),
                ("fc2.w", (self.classes, self.hidden)), ("fc2.b", (self.classes,))]

    def num_params(self) -> int:
        return sum(math.prod(s) for _, s in self.param_shapes())

    def flops_per_image(self) -> float:
        """Training FLOPs per image (forward x 3: one forward, two backward GEMM-shaped passes)."""
        s1, s2 = self.image - 2, self.image - 4
        fwd = 2 * (s1 * s1 * self.c1 * 9 + s2 * s2 * self.c2 * self.c1 * 9 + self.pooled * self.hidden
                   + self.hidden * self.classes)
        return 3.0 * fwd


_CONV_PARAMS = ("conv1.w", "conv1.b", "conv2.w", "conv2.b")


class _ConvStack(torch.autograd.Function):
    """conv1+ReLU -> conv2+ReLU -> 2x2 max-pool -> dropout through the HIP kernels; the backward
    writes the four conv gradients straight into the flat buffer (no autograd accumulation)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, model, step):
        from ..ops import fused

        hip = fused.hip()
        p_drop = model.cfg.p1 if model.training else 0.0
        x = x.reshape(x.shape[0], model.cfg.image, model.cfg.image)
        h1 = hip.mnist_conv1_fwd(x, w1.detach(), b1.detach())
        p, code = hip.mnist_conv2_pool_fwd(h1, w2.detach(), b2.detach(), step, model.drop_seed, p_drop)
        ctx.save_for_backward(x, h1, code)
        ctx.model, ctx.p_drop = model, p_drop
        return p.view(p.shape[0], -1)

    @staticmethod
    def backward(ctx, dp):
        from ..ops import fused

        x, h1, code = ctx.saved_tensors
        flat = ctx.model.flat
        w = [flat.params[n].detach() for n in _CONV_PARAMS]
        g = [flat.params[n].grad for n in _CONV_PARAMS]
        fresh = flat.direct["conv1.w"]
        fused.hip().mnist_conv_bwd(dp.contiguous(), code, x, h1, *w, *g, ctx.p_drop, not fresh)
        for n in _CONV_PARAMS:
            flat.mark_written(n)
        return None, None, None, None, None, None, None


_HEAD_PARAMS = ("fc1.w", "fc1.b", "fc2.w", "fc2.b")


class _Head(torch.autograd.Function):
    """fc1 -> ReLU -> dropout -> fc2 -> mean softmax cross-entropy.  Library GEMMs (bias in the
    epilogue) plus four HIP kernels (``relu_dropout`` fwd/bwd, ``xent10`` fwd/bwd) that also produce
    the bias gradients; weight gradients are GEMMs into the flat buffer (``mm(out=)``), so neither
    an AccumulateGrad add nor a zero fill runs."""

    @staticmethod
    def forward(ctx, feats, w1, b1, w2, b2, labels, model, step):
        from ..ops import fused

        hip = fused.hip()
        p_drop = model.cfg.p2 if model.training else 0.0
        w1, b1, w2, b2 = w1.detach(), b1.detach(), w2.detach(), b2.detach()
        h = torch.addmm(b1, feats, w1.t())
        h2, mask = hip.mnist_relu_dropout_fwd(h, step, model.drop_seed ^ 0x5BD1E995, p_drop)
        logits = torch.addmm(b2, h2, w2.t())
        loss, dlog = hip.mnist_xent10_fwd(logits, labels)
        ctx.save_for_backward(feats, h2, mask, dlog)
        ctx.model, ctx.p_drop = model, p_drop
        return loss

    @staticmethod
    def backward(ctx, g):
        from ..ops import fused

        hip = fused.hip()
        feats, h2, mask, dlog = ctx.saved_tensors
        flat = ctx.model.flat
        P = flat.params
        acc = not flat.direct["fc1.w"]
        dlogits = hip.mnist_xent10_bwd(dlog, g.float().reshape(1).contiguous(), P["fc2.b"].grad, acc)
        if acc:
            P["fc2.w"].grad.addmm_(dlogits.t(), h2)
        else:
            torch.mm(dlogits.t(), h2, out=P["fc2.w"].grad)
        dh2 = dlogits.mm(P["fc2.w"].detach())
        dh = hip.mnist_relu_dropout_bwd(dh2, mask, P["fc1.b"].grad, ctx.p_drop, acc)
        if acc:
            P["fc1.w"].grad.addmm_(dh.t(), feats)
        else:
            torch.mm(dh.t(), feats, out=P["fc1.w"].grad)
        dfeats = dh.mm(P["fc1.w"].detach())
        for n in _HEAD_PARAMS:
            flat.mark_written(n)
        return dfeats, None, None, None, None, None, None, None


class MnistCNN(torch.nn.Module):
    def __init__(self, cfg: MnistConfig = MnistConfig(), device="cuda", seed: int = 0, conv: str = "hip"):
        super().__init__()
        if conv not in ("hip", "torch"):
            raise ValueError("conv must be 'hip' or 'torch'")
        self.cfg = cfg
        self.param_ready: Optional[Callable[[str], None]] = None  # ZeRO-1 weight all-gather wait (dp.py)
        self.flat = FlatParams(cfg.param_shapes(), device)
        for n, p in self.flat.params.items():
            self.register_parameter(n.replace(".", "_"), p)
        dev = self.flat.data.device
        self.conv = conv if dev.type == "cuda" else "torch"
        if self.conv == "hip":
            for n in _CONV_PARAMS + _HEAD_PARAMS:  # gradients written by the HIP backward, not by autograd
                self.flat.mark_direct(n)
        # dropout of the HIP path: counter-based hash of (seed, step, element); ``step_counter`` is
        # the optimizer's device step count when set (graph mode), else a per-forward counter
        self.drop_seed = (seed * 0x9E3779B1 + 0x7F4A7C15) & 0xFFFFFFFF
        self.step_counter: Optional[torch.Tensor] = None
        self._own_step = torch.zeros(1, dtype=torch.float32, device=dev)
        g = torch.Generator(device=dev).manual_seed(seed)  # same seed + device type => identical replicas
        with torch.no_grad():
            for n, p in self.flat.params.items():  # PyTorch's default conv/linear init: U(+-1/sqrt(fan_in))
                w = self.flat.shapes[n.split(".")[0] + ".w"]
                bound = 1.0 / math.sqrt(math.prod(w[1:]))
                p.copy_((torch.rand(p.shape, generator=g, device=dev) * 2 - 1) * bound)
            # class prototypes: smooth random strokes in [0, 1] (a 7x7 field upsampled to 28x28)
            coarse = torch.rand((cfg.classes, 1, 7, 7), generator=g, device=dev)
            proto = F.interpolate(coarse, size=(cfg.image, cfg.image), mode="bilinear", align_corners=False)
            proto = (proto > 0.6).float() * proto
        self.register_buffer("prototypes", proto, persistent=False)

    def P(self, name: str) -> torch.nn.Parameter:
        if self.param_ready is not None:
            self.param_ready(name)
        return self.flat.params[name]

    def synthetic_batch(self, batch: int, gen: Optional[torch.Generator] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """(images [B,1,28,28] normalised bf16 channels-last, labels [B] int64) on the model's device.
        ``gen=None`` draws from the device's default generator (hipGraph-capturable)."""
        dev = self.prototypes.device
        y = torch.randint(0, self.cfg.classes, (batch,), generator=gen, device=dev)
        noise = torch.randn((batch, 1, self.cfg.image, self.cfg.image), generator=gen, device=dev)
        x = (self.prototypes.index_select(0, y) + self.cfg.noise * noise - _MEAN) / _STD
        return x.to(self.flat.data.dtype).contiguous(memory_format=torch.channels_last), y

    def synthetic_batch_dev(self, batch: int, step: torch.Tensor, seed: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        """The same kind of batch from one HIP launch (``mnist_synth``), indexed by the device step
        counter ``step`` (fp32 [1], the optimizer's): a captured graph draws a new batch per replay."""
        from ..ops import fused

        x, y = fused.hip().mnist_synth(self.prototypes, int(batch), step, int(seed) & 0xFFFFFFFF, self.cfg.noise, _MEAN, _STD)
        return x.contiguous(memory_format=torch.channels_last), y

    def dropout_step(self) -> torch.Tensor:
        if self.step_counter is not None:
            return self.step_counter
        self._own_step.add_(1.0)
        return self._own_step

    def conv_features(self, x: torch.Tensor, step: Optional[torch.Tensor] = None) -> torch.Tensor:
        """[B,1,28,28] -> pooled features [B, 9216] in NHWC order (fc1's input).  ``step``: the
        dropout counter value of this forward (drawn here when not given)."""
        c = self.cfg
        if self.conv == "hip" and x.is_cuda:
            return _ConvStack.apply(x, *(self.P(n) for n in _CONV_PARAMS), self,
                                    step if step is not None else self.dropout_step())
        w1 = self.P("conv1.w").permute(0, 3, 1, 2)  # channels-last storage -> OIHW
        w2 = self.P("conv2.w").permute(0, 3, 1, 2)
        h = F.relu(F.conv2d(x, w1, self.P("conv1.b")))
        h = F.relu(F.conv2d(h, w2, self.P("conv2.b")))
        h = F.dropout(F.max_pool2d(h, 2), c.p1, self.training)
        return h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)

    def forward(self, x: torch.Tensor, labels: Optional[torch.Tensor] = None) -> torch.Tensor:
        c = self.cfg
        if self.conv == "hip" and x.is_cuda and labels is not None:
            step = self.dropout_step()
            feats = self.conv_features(x, step)
            return _Head.apply(feats, *(self.P(n) for n in _HEAD_PARAMS), labels, self, step)
        h = self.conv_features(x)
        h = F.dropout(F.relu(F.linear(h, self.P("fc1.w"), self.P("fc1.b"))), c.p2, self.training)
        logits = F.linear(h, self.P("fc2.w"), self.P("fc2.b"))
        if labels is None:
            return logits
        return F.cross_entropy(logits.float(), labels)


def _mix32(x):
    import numpy as np

    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def synth_reference(prototypes: torch.Tensor, batch: int, step: int, seed: int, cfg: MnistConfig = MnistConfig()):
    """numpy/fp32 reference of the ``mnist_synth`` HIP kernel (the numerics test compares them)."""
    import numpy as np

    with np.errstate(over="ignore"):
        proto = prototypes.detach().float().cpu().numpy().reshape(prototypes.shape[0], -1)
        classes, pixels = proto.shape
        u = lambda v: np.asarray(v, dtype=np.uint32)  # noqa: E731
        h3 = lambda a, b, c: _mix32(u(a) ^ _mix32(u(b) ^ _mix32(u(c))))  # noqa: E731
        b = np.arange(batch, dtype=np.uint32)
        y = (h3(seed, step, u(0x9E3779B9) ^ b) % u(classes)).astype(np.int64)
        p = np.arange(0, pixels, 2, dtype=np.uint32)
        idx = b[:, None] * u(pixels) + p[None, :]
        h1 = h3(u(seed) ^ u(0x85EBCA6B), step, idx)
        h2 = _mix32(h1 ^ u(0x27D4EB2F))
        u1 = ((h1 >> u(8)) + u(1)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        u2 = (h2 >> u(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        r = np.sqrt(np.float32(-2.0) * np.log(u1))
        a = np.float32(6.28318530718) * u2
        z = np.stack([r * np.cos(a), r * np.sin(a)], axis=-1).reshape(batch, -1)[:, :pixels]
        x = (proto[y] + np.float32(cfg.noise) * z - np.float32(_MEAN)) / np.float32(_STD)
    side = int(round(pixels ** 0.5))
    return torch.from_numpy(x.astype(np.float32)).view(batch, 1, side, side), torch.from_numpy(y)
