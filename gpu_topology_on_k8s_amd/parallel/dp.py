"""Data parallelism over RCCL/xGMI on the scheduler-chosen devices (DP row).

One process per GPU.  Gradients live in one flat bf16 buffer (:class:`~..models.llama.FlatParams`);
:class:`BucketedAllReduce` cuts it into contiguous buckets in *reverse* parameter order (the order
backward produces them), and each parameter's post-accumulate-grad hook counts down its bucket: the
moment a bucket is complete its ``all_reduce`` is issued asynchronously on RCCL's stream, overlapping
the rest of backward.

Bucket size is chosen for xGMI, not NVSwitch: an MI355X ring all-reduce is per-link bound (one
≈153 GB/s link per neighbour pair), and RCCL reaches its plateau bus bandwidth only for messages in
the hundreds of MB, so the default is 256 MiB buckets (≈64 collectives for Llama-3-8B's 16 GB of
gradients) instead of DDP's 25 MB — fewer, larger collectives, with the 288 GB HBM making the
bucket memory irrelevant.  The first bucket to complete is sized smaller (``first_bucket_mb``) so
communication starts early.  Parameters are broadcast from rank 0 at start (C3).

``zero1=True`` shards the optimizer (ZeRO stage 1) over the same buckets: each bucket is
reduce-scattered instead of all-reduced (rank r receives the summed chunk r of every bucket, in
place), the optimizer updates only those chunks (:meth:`shards`), and :meth:`gather_params`
all-gathers the updated bf16 weights bucket by bucket, in forward order, asynchronously.  The next
forward waits per bucket (:meth:`wait_param`, installed as ``Llama.param_ready``), so the all-gather
of late layers overlaps the compute of early ones.  Communication volume equals the all-reduce's;
fp32 master/m/v memory and AdamW time drop by the world size (96 GB -> 12 GB per GPU for
Llama-3-8B on 8 GPUs).  Every bucket is a whole number of 64-element-aligned parameters, so its
length splits into 8-element-multiple chunks for any world size up to 8.

``grad_reduce="fp32"`` reduces each bucket in fp32 (a widened copy in :attr:`grad32`, all-reduced or
reduce-scattered there) and the optimizer reads that fp32 sum: the averaged gradient is rounded to
bf16 nowhere, against the bf16 ring whose partial sums round at every hop.  It doubles the bytes
on the links; bf16 stays the default (tests/test_llama_dp_cpu.py measures both against an exact sum).

``comm_ctas`` caps the CTAs (CUs) RCCL may use per collective (``ncclConfig_t.maxCTAs`` through the
process group's options, :func:`nccl_options`): during backward the collectives share the GPU with
hipBLASLt's GEMMs, which hold every CU.  :class:`CommShadow` measures that contention on one GPU
(profiles/r04_comm_shadow): a GEMM that shares even a few CUs with a collective runs at the pace
of its slowest CU, so the step pays for *how long* any CU is shared, not for how many are.  Too few
CTAs stretch each collective past its link-rate duration (16 CTAs: 3x, +14 % step time); too many
share every CU (256: +7.7 %).  :data:`DEFAULT_COMM_CTAS` = 64 is the knee at 250-350 GB/s bus
bandwidth for Llama-3-8B's 67 buckets per step (+4.4 % / +5.9 %).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["BucketedAllReduce", "Bucket", "broadcast_params", "CommShadow", "DEFAULT_COMM_CTAS", "nccl_options", "ring_bytes"]

# RCCL CTAs per DP collective (profiles/r04_comm_shadow/SUMMARY.md)
DEFAULT_COMM_CTAS = 64


def nccl_options(max_ctas: int = 0, min_ctas: int = 0):
    """``ProcessGroupNCCL.Options`` with RCCL's CTA bounds (``ncclConfig_t`` minCTAs / maxCTAs); ``None``
    when both are 0 (RCCL's own choice)."""
    if not (max_ctas or min_ctas):
        return None
    o = dist.ProcessGroupNCCL.Options()
    if max_ctas:
        o.config.max_ctas = int(max_ctas)
    if min_ctas:
        o.config.min_ctas = int(min_ctas)
    return o


def ring_bytes(nbytes: int, k: int) -> int:
    """Bytes each member of a k-rank ring all-reduce sends (and receives): 2 (k-1)/k of the message."""
    return int(nbytes * 2 * (k - 1) / k) if k > 1 else 0


class CommShadow:
    """The collective a k-GPU DP step would run for each gradient bucket, played on one GPU
    (VERDICT r3 next #4): ``ctas`` workgroups (RCCL's CTAs) copy the bucket's ring traffic through
    local HBM, paced over the collective's duration ``ring_bytes / busbw`` on a side stream, from the
    bucket-ready hook, exactly where the real all-reduce would start (csrc/ops/comm_shadow.hip).  The
    compute stream waits for it before the optimizer, as it waits for RCCL."""

    def __init__(self, device, ctas: int, k: int = 8, busbw_gbps: float = 350.0, max_bucket_bytes: int = 256 << 20):
        self.ctas, self.k, self.busbw = int(ctas), int(k), float(busbw_gbps)
        nb = max(16, ring_bytes(max_bucket_bytes, self.k))
        self.src = torch.empty(nb, dtype=torch.uint8, device=device)
        self.dst = torch.empty(nb, dtype=torch.uint8, device=device)
        self.stream = torch.cuda.Stream(device=device)
        self.launched = 0
        self.bytes = 0
        self.micros = 0.0
        # per step: the (start, end) events of every collective and the compute stream's event at the
        # point where it starts waiting for them (timing(): achieved durations and the exposed tail)
        self.steps: List[Tuple[object, List[Tuple[object, object]]]] = []
        self._cur: List[Tuple[object, object]] = []

    def launch(self, bucket_bytes: int, part: str = "ar"):
        """Play one bucket's collective: ``ar`` the all-reduce (2 (k-1)/k of the bucket through each
        rank); under ZeRO-1 ``rs`` the reduce-scatter at the bucket hook and ``ag`` the weight
        all-gather after the optimizer, (k-1)/k each.  Returns the collective's end event."""
        from ..ops import fused

        nb = ring_bytes(bucket_bytes, self.k)
        if part in ("rs", "ag"):
            nb //= 2
        nb = min(nb, self.src.numel())
        us = nb / (self.busbw * 1e9) * 1e6
        cur = torch.cuda.current_stream(self.src.device)
        self.stream.wait_stream(cur)  # the bucket's gradients are complete
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.stream):
            ev0.record(self.stream)
            fused.hip().comm_shadow(self.src, self.dst, nb, self.ctas, us)
            ev1.record(self.stream)
        self._cur.append((ev0, ev1))
        self.launched += 1
        self.bytes += nb
        self.micros += us
        return ev1

    def wait(self) -> None:
        cur = torch.cuda.current_stream(self.src.device)
        ready = torch.cuda.Event(enable_timing=True)
        ready.record(cur)
        cur.wait_stream(self.stream)
        if self._cur:
            self.steps.append((ready, self._cur))
            self._cur = []
            if len(self.steps) > 64:  # a long run keeps the last 64 steps' events, not every step's
                del self.steps[0]

    def reset_timing(self) -> None:
        self.steps, self._cur = [], []

    def timing(self) -> Dict[str, float]:
        """Per step, averaged over the steps since reset_timing(): the summed collective kernel time
        (target: the sum of ring_bytes / busBW; more means N CTAs could not move the bytes in time)
        and the exposed tail, from the compute stream reaching the optimizer to the last collective's
        end (what overlap could not hide)."""
        if not self.steps:
            return {"achieved_ms_per_step": 0.0, "exposed_ms_per_step": 0.0, "steps_timed": 0}
        torch.cuda.synchronize(self.src.device)
        ach = exp = 0.0
        for ready, evs in self.steps:
            ach += sum(a.elapsed_time(b) for a, b in evs)
            exp += max(0.0, ready.elapsed_time(evs[-1][1]))
        n = len(self.steps)
        return {"achieved_ms_per_step": ach / n, "exposed_ms_per_step": exp / n, "steps_timed": n}


@dataclass
class Bucket:
    index: int
    start: int  # element offsets into the flat grad buffer
    end: int
    params: List[str] = field(default_factory=list)
    pending: int = 0
    work: Optional[object] = None
    gather_work: Optional[object] = None
    gather_event: Optional[object] = None  # one-GPU comm shadow of the ZeRO-1 all-gather
    launched_at: float = 0.0

    @property
    def numel(self) -> int:
        return self.end - self.start


def broadcast_params(flat, group=None, src: int = 0) -> None:
    """Rank ``src`` -> everyone (ncclBroadcast of the whole flat parameter buffer, C3)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(flat.data, src=src, group=group)
    if hasattr(flat, "invalidate_t"):
        flat.invalidate_t()  # persistent W^T (models/llama.py) is re-made from the broadcast weights


class BucketedAllReduce:
    def __init__(self, flat, group=None, bucket_mb: float = 256.0, first_bucket_mb: float = 64.0, average: bool = True,
                 overlap: bool = True, zero1: bool = False, grad_reduce: str = "bf16",
                 shadow: Optional[CommShadow] = None):
        if grad_reduce not in ("bf16", "fp32"):
            raise ValueError("grad_reduce must be 'bf16' or 'fp32'")
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.zero1 = zero1
        self.average = average
        self.overlap = overlap
        esz = flat.grad.element_size()
        cap = max(1, int(bucket_mb * (1 << 20) / esz))
        first_cap = min(cap, max(1, int(first_bucket_mb * (1 << 20) / esz)))  # never larger than the others
        # Parameters sit in the flat buffer in registration order, so reverse registration order
        # (the order backward finishes gradients) walks the buffer downwards and every bucket is
        # one contiguous range.  Bucket 0 (the first to complete) is capped smaller.
        self.buckets: List[Bucket] = []
        self.bucket_of: Dict[str, int] = {}
        cur: Optional[Bucket] = None
        for n in reversed(flat.names):
            s, e = flat.span(n)
            limit = first_cap if len(self.buckets) <= 1 and cur is not None and cur.index == 0 else cap
            if cur is None or (cur.params and cur.numel + (e - s) > limit):
                cur = Bucket(index=len(self.buckets), start=s, end=e)
                self.buckets.append(cur)
            cur.start = min(cur.start, s)
            cur.params.append(n)
            self.bucket_of[n] = cur.index
        # tile the whole buffer (alignment padding between params is zero and stays zero)
        for i, b in enumerate(self.buckets):
            b.end = flat.numel if i == 0 else self.buckets[i - 1].start
        if self.buckets:
            self.buckets[-1].start = 0
        self._hooks = []
        if zero1:
            # every rank's chunk must be a multiple of 8 elements (the fused AdamW / norm kernels' vector width)
            bad = [b.index for b in self.buckets if b.numel % (8 * self.world)]
            if bad:
                raise ValueError(f"zero1: buckets {bad[:4]} do not split into 8-element chunks over {self.world} ranks")
        self.stats = {"buckets": len(self.buckets), "bucket_mb": bucket_mb, "launches": 0, "comm_bytes": 0,
                      "zero1": zero1, "grad_reduce": grad_reduce}
        # fp32 reduction: the buckets are widened into this buffer and reduced there; the optimizer
        # reads it (reduced_grad).  Only at world > 1: one rank has nothing to sum.
        self.grad_reduce = grad_reduce
        self.grad32 = (torch.zeros(flat.numel, dtype=torch.float32, device=flat.grad.device)
                       if grad_reduce == "fp32" and self.world > 1 else None)
        self.shadow = shadow if (shadow is not None and self.world == 1 and flat.grad.is_cuda) else None
        # (A per-bucket clipping norm on a side stream as buckets land measured flat on MI355X --
        # hipBLASLt's GEMMs hold every CU -- and was retired in round 5: profiles/r01_fuse_res/NORM.md.)
        self._launched = [False] * len(self.buckets)
        # reduction check (capture_local / verify): each bucket's local gradient as its collective saw it
        self.snapshot: Optional[torch.Tensor] = None
        self._capture = False
        self._suspended = False
        if overlap and (self.world > 1 or self.shadow is not None):
            direct = getattr(flat, "direct", {})
            for n, p in flat.params.items():
                if n in direct:  # weight-gradient GEMM writes the flat buffer itself (models/llama.py _FlatLinear)
                    self._hooks.append(flat.add_ready_hook(n, self._make_hook(n)))
                else:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(n)))
        self.reset()

    def _make_hook(self, name: str):
        def hook(p: torch.Tensor) -> None:
            if self._suspended:
                return
            b = self.buckets[self.bucket_of[name]]
            b.pending -= 1
            if b.pending == 0:
                self._launch(b)

        return hook

    def own(self, b: Bucket):
        """Element range of bucket ``b`` this rank owns under zero1 (the whole bucket otherwise)."""
        if not self.zero1:
            return b.start, b.end
        c = b.numel // self.world
        return b.start + self.rank * c, b.start + (self.rank + 1) * c

    def shards(self) -> List[tuple]:
        """The flat-buffer ranges this rank's optimizer updates, in buffer order."""
        return sorted(self.own(b) for b in self.buckets)

    def _launch(self, b: Bucket) -> None:
        self._launched[b.index] = True
        if self.world == 1:  # nothing to reduce: only the k-GPU shadow
            if self.shadow is not None:
                self.shadow.launch(b.numel * self.flat.grad.element_size(), "rs" if self.zero1 else "ar")
            return
        view = self.flat.grad[b.start:b.end]
        b.launched_at = time.perf_counter()
        if self._capture:  # the exact input of this bucket's collective, copied on the launching stream
            self.snapshot[b.start:b.end].copy_(view)
        if self.grad32 is not None:  # widen, then reduce in fp32
            buf = self.grad32[b.start:b.end]
            buf.copy_(view)
            view = buf
        src = self.grad32 if self.grad32 is not None else self.flat.grad
        if self.zero1:
            s, e = self.own(b)
            b.work = dist.reduce_scatter_tensor(src[s:e], view, group=self.group, async_op=True)
        else:
            b.work = dist.all_reduce(view, group=self.group, async_op=True)
        self.stats["launches"] += 1
        self.stats["comm_bytes"] += view.numel() * view.element_size()

    # ---------------------------------------------------------------- reduction check
    def suspend(self, on: bool) -> None:
        """While suspended the readiness hooks launch nothing (a hook-free backward: the local gradient
        of models/train.py's --check-reduction reference pass); leaving suspension resets the counts."""
        self._suspended = bool(on)
        if not on:
            self.reset()

    def capture_local(self, on: bool) -> None:
        """While on, each bucket's local gradient is copied into :attr:`snapshot` on the launching
        stream right before its collective is issued: exactly what that collective reduced."""
        if on and self.snapshot is None:
            self.snapshot = torch.zeros_like(self.flat.grad)
        self._capture = bool(on)

    def reduced_buffer(self) -> torch.Tensor:
        """The buffer the optimizer reads after :meth:`finish` (fp32 under ``grad_reduce="fp32"``)."""
        return self.grad32 if self.grad32 is not None else self.flat.grad

    def freeze(self) -> torch.Tensor:
        """A copy of the buffer the optimizer reads, taken on the current stream at the point the
        optimizer reads it and before any verification collective: on RCCL those collectives run on
        the communicator's stream behind the reductions, and a read after them would hide a reduction
        the optimizer never waited for.  Host memory (pinned) for a GPU buffer."""
        src = self.reduced_buffer()
        if not src.is_cuda:
            return src.clone()
        out = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        out.copy_(src, non_blocking=True)
        torch.cuda.current_stream(src.device).synchronize()
        return out

    def _gather(self, x: torch.Tensor) -> List[torch.Tensor]:
        if self.world == 1:
            return [x]
        raw = x.contiguous()
        if raw.dtype not in (torch.float32, torch.float64):  # bit-exact through any backend (gloo has no bf16)
            raw = raw.view(torch.uint8)
        parts = [torch.empty_like(raw) for _ in range(self.world)]
        dist.all_gather(parts, raw, group=self.group)
        return [q.view(x.dtype) for q in parts]

    def verify(self, local: torch.Tensor, against: Optional[torch.Tensor] = None,
               frozen: Optional[torch.Tensor] = None) -> Dict[str, object]:
        """Per bucket: the reduced gradient the optimizer reads (this rank's own range under zero1)
        against the exact sum over ranks of ``local`` -- every rank's local gradient, all-gathered
        bit-exactly and summed in fp64.  ``against``: compare with this buffer instead of the
        reduced one, rank-locally (``snapshot`` vs a hook-free pass: was each bucket complete when its
        collective launched?).  ``frozen``: the reduced buffer as :meth:`freeze` took it (else it is
        read now).  -> ``{"max_rel": worst relative L2 error, "buckets": [...]}``."""
        out, worst = [], 0.0
        for b in self.buckets:
            s, e = self.own(b)
            if against is None:
                parts = self._gather(local[b.start:b.end])
                exact = torch.zeros(e - s, dtype=torch.float64, device=local.device)
                for q in parts:
                    exact += q[s - b.start:e - b.start].double()
                got = (frozen[s:e].to(exact.device) if frozen is not None else self.reduced_buffer()[s:e]).double()
            else:  # the whole bucket: every rank's snapshot holds its own local bucket
                exact = local[b.start:b.end].double()
                got = against[b.start:b.end].double()
            den = float(exact.norm())
            err = float((got - exact).norm())
            rel = err / den if den > 0 else err
            worst = max(worst, rel)
            out.append({"index": b.index, "rel": rel})
        return {"max_rel": worst, "buckets": out}

    def reset(self) -> None:
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
        self._launched = [False] * len(self.buckets)

    def finish(self) -> None:
        """After ``loss.backward()``: launch stragglers (params without grads), wait for everything."""
        if hasattr(self.flat, "fill_unwritten"):
            self.flat.fill_unwritten()  # a direct gradient nobody wrote this step is zero, not stale
        if self.world > 1:
            for b in self.buckets:
                if b.work is None:
                    self._launch(b)
            for b in self.buckets:
                b.work.wait()
        elif self.shadow is not None:
            for b in self.buckets:
                if not self._launched[b.index]:
                    self._launch(b)
            if self.shadow is not None:
                self.shadow.wait()  # the optimizer waits for the (shadow) collectives, as for RCCL's
        self.reset()

    @property
    def reduced_grad(self) -> Optional[torch.Tensor]:
        """The fp32 reduced gradient the optimizer reads under ``grad_reduce="fp32"`` (None: the flat bf16
        gradient buffer holds the reduced gradient)."""
        return self.grad32

    def gather_params(self) -> None:
        """zero1, after the optimizer step: all-gather every bucket's updated weights, asynchronously,
        first-used bucket (highest index: the embedding end of the buffer) first."""
        if self.zero1 and self.world == 1 and self.shadow is not None:
            for b in reversed(self.buckets):  # the k-GPU job's all-gathers, played on the shadow stream
                b.gather_event = self.shadow.launch(b.numel * self.flat.data.element_size(), "ag")
            return
        if not self.zero1 or self.world == 1:
            return
        for b in reversed(self.buckets):
            s, e = self.own(b)
            b.gather_work = dist.all_gather_into_tensor(self.flat.data[b.start:b.end], self.flat.data[s:e], group=self.group,
                                                        async_op=True)

    def wait_param(self, name: str) -> None:
        """Forward pre-use hook: the current stream waits for the all-gather of ``name``'s bucket."""
        b = self.buckets[self.bucket_of[name]]
        if b.gather_work is not None:
            b.gather_work.wait()
            b.gather_work = None
        if b.gather_event is not None:
            torch.cuda.current_stream(self.flat.data.device).wait_event(b.gather_event)
            b.gather_event = None

    def wait_all_params(self) -> None:
        for b in self.buckets:
            if b.gather_work is not None:
                b.gather_work.wait()
                b.gather_work = None
            if b.gather_event is not None:
                torch.cuda.current_stream(self.flat.data.device).wait_event(b.gather_event)
                b.gather_event = None

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world if self.average else 1.0

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
