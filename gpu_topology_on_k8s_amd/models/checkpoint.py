"""Training checkpoints for the flat-buffer Llama: asynchronous sharded save, reshardable resume.

The reference has no training loop; its only persisted state is the scheduler's pod/node
annotations.  The config-5 workload (``models/train.py``) is a real multi-hour DP
job on the devices the extender placed it on, so it needs the usual save/resume:

    <dir>/step_000100/meta.json                 step, Adam t, flat layout, world, zero1   (rank 0)
    <dir>/step_000100/state_rank{r}.safetensors "flat" (bf16 weights), "master"/"m"/"v" (fp32):
                                                the concatenation of the rank's flat ranges,
                                                "shards": int64 [n, 2] = those ranges
    <dir>/step_000100/rng_rank{r}.safetensors   the rank's data-generator state
    <dir>/latest                                name of the newest committed step directory

Layout choices for MI355X:

- **One tensor per state, not one per parameter.**  Parameters, gradients and the AdamW state are
  single flat buffers already (``FlatParams``, ``FlatAdamW``), so a save is three or four large
  device→host copies — HBM→PCIe streams at full rate — instead of ~300 small ones.
- **Asynchronous.**  The copies go to pinned host buffers (allocated once, reused) on a side HIP
  stream; the compute stream waits on an event, not the host, so the next optimizer step cannot
  overwrite state being copied.  A writer thread then serialises to safetensors while training
  continues.  The commit (barrier, ``meta.json``, rename, ``latest``) runs on the main thread at the
  next :meth:`CheckpointWriter.save` or :meth:`CheckpointWriter.close`, so no collective is ever
  issued from the writer thread.
- **Every rank writes 1/W.**  With ``--zero1`` each rank writes the weights and fp32 state of its
  own shards; without it the (replicated) state is split into W contiguous ranges, one per rank.
  Either way a rank writes ~14 B x params / W (14 GB per GPU for Llama-3-8B at W=8) — no single
  112 GB writer.
- **Reshardable.**  Every optimizer file records the flat ranges it holds, and resume reads
  exactly the ranges the *new* layout owns (``safe_open(...).get_slice``, no full loads), so a job
  can resume on a different world size or switch ZeRO-1 on or off — what happens when the extender
  re-places a restarted pod on a different k.

Nothing is unpickled: safetensors and JSON only.
"""
from __future__ import annotations

import json
import os
import shutil
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from safetensors import safe_open

__all__ = ["CheckpointWriter", "write_safetensors", "read_ranges", "load_checkpoint", "latest_checkpoint", "read_optimizer_ranges"]

FORMAT = 2


_ST_DTYPES = {torch.float32: "F32", torch.bfloat16: "BF16", torch.float16: "F16", torch.int64: "I64",
              torch.int32: "I32", torch.uint8: "U8", torch.int8: "I8"}
_ST_NAMES = {v: k for k, v in _ST_DTYPES.items()}


def write_safetensors(path: str, tensors: Dict[str, torch.Tensor]) -> None:
    """Write a safetensors file straight from (pinned) host memory.

    ``safetensors.torch.save_file`` first materialises every tensor as a Python ``bytes`` object —
    a second full host copy of tens of GB, built while holding the GIL.  Here the header is JSON
    and each tensor is handed to ``write`` as a zero-copy memoryview, so the writer thread spends
    its time in the syscall with the GIL released and the training loop keeps running.
    """
    header, off, order = {}, 0, []
    for name in sorted(tensors):
        t = tensors[name].contiguous()
        if t.device.type != "cpu":
            raise ValueError(f"{name}: host tensor expected")
        n = t.numel() * t.element_size()
        header[name] = {"dtype": _ST_DTYPES[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + n]}
        order.append(t)
        off += n
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * (-len(hb) % 8)
    with open(path, "wb") as f:
        f.write(len(hb).to_bytes(8, "little"))
        f.write(hb)
        for t in order:
            if t.numel():
                f.write(memoryview(t.reshape(-1).view(torch.uint8).numpy()))


def _concat_offsets(shards) -> List[Tuple[int, int, int]]:
    """(start, end, offset in the concatenation) for each shard."""
    out, o = [], 0
    for a, b in shards:
        out.append((a, b, o))
        o += b - a
    return out


def _to_concat(base, s: int) -> int:
    for a, b, o in base:
        if a <= s < b:
            return o + s - a
    raise ValueError(f"flat offset {s} is not in this rank's shards")


def _rank_world() -> Tuple[int, int]:
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _layout(flat) -> List[list]:
    return [[n, int(flat.offsets[n]), list(flat.shapes[n])] for n in flat.names]


def latest_checkpoint(root: str) -> Optional[str]:
    """The newest committed step directory under ``root`` (``None`` if there is none).

    ``latest`` names it; if that directory is incomplete (a crash while an existing step was being
    replaced), the step's moved-aside ``.step_N.old`` or else the newest complete ``step_N`` is used."""
    p = os.path.join(root, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        name = f.read().strip()
    for d in (os.path.join(root, name), os.path.join(root, f".{name}.old")):
        if os.path.exists(os.path.join(d, "meta.json")):
            return d
    done = sorted((x for x in os.listdir(root) if x.startswith("step_") and x[5:].isascii() and x[5:].isdigit()
                   and os.path.exists(os.path.join(root, x, "meta.json"))), key=lambda x: int(x[5:]))
    return os.path.join(root, done[-1]) if done else None


class CheckpointWriter:
    """Asynchronous checkpoint writer for one rank (every rank constructs one)."""

    def __init__(self, root: str, model, opt, model_name: str = "", keep: int = 2, zero1: bool = False):
        self.root, self.model, self.opt = root, model, opt
        self.model_name, self.keep, self.zero1 = model_name, keep, zero1
        self.rank, self.world = _rank_world()
        self._pinned: Dict[str, torch.Tensor] = {}
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None
        self._pending: Optional[Tuple[int, str]] = None  # (step, tmp dir) awaiting commit
        self._stream = None
        self.saved: List[int] = []
        # host-side cost of save() (snapshot issue), commit wait, background write time and bytes
        self.stats = {"saves": 0, "snapshot_ms": 0.0, "commit_wait_ms": 0.0, "write_s": 0.0, "bytes": 0}
        os.makedirs(root, exist_ok=True)

    # -- snapshot ------------------------------------------------------------------------------
    def write_ranges(self) -> List[Tuple[int, int]]:
        """The flat-buffer ranges this rank writes: its ZeRO-1 shards, or (replicated state) a 1/W
        contiguous slice, so every rank writes ~(2 + 12) B x params / W and no rank is the 112 GB
        single writer of an 8 B-parameter model."""
        if self.opt.sharded:
            return [tuple(r) for r in self.opt.shards]
        n = self.model.flat.numel
        chunk = -(-n // (self.world * 8)) * 8
        s, e = min(n, self.rank * chunk), min(n, (self.rank + 1) * chunk)
        return [(s, e)] if e > s else []

    def _gather(self, key: str, src: torch.Tensor, ranges, base) -> torch.Tensor:
        """Device->host copy of ``src``'s ``ranges`` (concatenated) into a reused pinned buffer.
        ``base`` maps a flat offset to ``src``'s index: 0 for the flat buffer, else the shard
        concatenation offsets of the optimizer state."""
        total = sum(e - s for s, e in ranges)
        if src.is_cuda:
            buf = self._pinned.get(key)
            if buf is None or buf.numel() != total or buf.dtype != src.dtype:
                buf = torch.empty(total, dtype=src.dtype, pin_memory=True)
                self._pinned[key] = buf
        else:
            buf = torch.empty(total, dtype=src.dtype)
        o = 0
        for s, e in ranges:
            i = s if base == 0 else _to_concat(base, s)
            buf[o:o + e - s].copy_(src[i:i + e - s], non_blocking=src.is_cuda)
            o += e - s
        return buf

    def prepare(self) -> None:
        """Allocate the pinned host buffers now (pinning tens of GB takes ~1 s), e.g. before a
        timed loop, instead of inside the first save."""
        if not self.model.flat.data.is_cuda:
            return
        total = sum(e - s for s, e in self.write_ranges())
        for k, t in (("flat", self.model.flat.data), ("master", self.opt.master), ("m", self.opt.m), ("v", self.opt.v)):
            if k not in self._pinned:
                self._pinned[k] = torch.empty(total, dtype=t.dtype, pin_memory=True)

    def _snapshot(self, gen: Optional[torch.Generator]) -> Tuple[Dict[str, Dict[str, torch.Tensor]], Optional[torch.cuda.Event]]:
        flat, opt = self.model.flat, self.opt
        files: Dict[str, Dict[str, torch.Tensor]] = {}
        dev = flat.data.device
        ev = None
        if dev.type == "cuda":
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=dev)
            cur = torch.cuda.current_stream(dev)
            self._stream.wait_stream(cur)
            ctx = torch.cuda.stream(self._stream)
        else:
            ctx = _nullctx()
        ranges = self.write_ranges()
        with ctx:
            st = {"flat": self._gather("flat", flat.data, ranges, 0)}
            # optimizer state is stored as the concatenation of opt.shards; map ranges into it
            base = _concat_offsets(opt.shards)
            for k in ("master", "m", "v"):
                st[k] = self._gather(k, getattr(opt, k), ranges, base)
            st["shards"] = torch.tensor(ranges, dtype=torch.int64).reshape(-1, 2)
            files[f"state_rank{self.rank}.safetensors"] = st
        if dev.type == "cuda":
            ev = torch.cuda.Event()
            ev.record(self._stream)
            # Only the optimizer step (and the ZeRO-1 all-gather after it) writes weights or
            # state, so the compute stream waits on the copy there: the next forward/backward
            # overlaps the device->host DMA instead of queueing behind it.
            opt.defer_until(ev)
        if gen is not None:
            files[f"rng_rank{self.rank}.safetensors"] = {"rng": gen.get_state().clone()}
        return files, ev

    # -- save / commit -------------------------------------------------------------------------
    def save(self, step: int, gen: Optional[torch.Generator] = None, blocking: bool = False) -> None:
        """Snapshot the state after ``step`` optimizer steps and write it in the background.

        The previous save (if any) is committed first.  ZeRO-1 callers must have waited for the
        weight all-gather (``BucketedAllReduce.wait_all_params``) before saving.
        """
        self._commit()
        t0 = time.perf_counter()
        tmp = os.path.join(self.root, f".step_{step:06d}.tmp")
        if self.rank == 0:
            shutil.rmtree(tmp, ignore_errors=True)
            os.makedirs(tmp)
        if dist.is_initialized():
            dist.barrier()
        files, ev = self._snapshot(gen)
        meta = {
            "format": FORMAT, "step": int(step), "adam_t": int(self.opt.t), "numel": int(self.model.flat.numel),
            "world": self.world, "zero1": bool(self.zero1), "model": self.model_name, "layout": _layout(self.model.flat),
            "hyper": {"lr": self.opt.lr, "betas": list(self.opt.betas), "eps": self.opt.eps, "wd": self.opt.wd,
                      "clip_norm": self.opt.clip_norm},
        }

        nbytes = sum(t.numel() * t.element_size() for ts in files.values() for t in ts.values())

        def write():
            try:
                w0 = time.perf_counter()
                if ev is not None:
                    ev.synchronize()
                for name, tensors in files.items():
                    write_safetensors(os.path.join(tmp, name), tensors)
                self.stats["write_s"] += time.perf_counter() - w0
                self.stats["bytes"] += nbytes
                if self.rank == 0:
                    with open(os.path.join(tmp, "meta.part.json"), "w") as f:
                        json.dump(meta, f)
            except BaseException as e:  # surfaced on the main thread at commit
                self._error = e

        self._pending = (step, tmp)
        self._thread = threading.Thread(target=write, name=f"ckpt-{step}", daemon=True)
        self._thread.start()
        self.stats["saves"] += 1
        self.stats["snapshot_ms"] += (time.perf_counter() - t0) * 1e3
        if blocking:
            self._commit()

    def _commit(self) -> None:
        if self._pending is None:
            return
        step, tmp = self._pending
        self._pending = None
        t0 = time.perf_counter()
        self._thread.join()
        self.stats["commit_wait_ms"] += (time.perf_counter() - t0) * 1e3
        self._thread = None
        ok = torch.tensor([0 if self._error is not None else 1], dtype=torch.int32)
        if dist.is_initialized():
            if dist.get_backend() == "nccl":
                ok = ok.cuda()
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) != 1:
            err, self._error = self._error, None
            raise RuntimeError(f"checkpoint step {step} failed on a rank") from err
        if self.rank == 0:
            final = os.path.join(self.root, f"step_{step:06d}")
            os.replace(os.path.join(tmp, "meta.part.json"), os.path.join(tmp, "meta.json"))
            # re-saving an existing step (a resumed run): move the old directory aside first, so a
            # crash at any point leaves `latest` naming a complete directory (old or new)
            old = None
            if os.path.exists(final):
                old = os.path.join(self.root, f".step_{step:06d}.old")
                shutil.rmtree(old, ignore_errors=True)
                os.replace(final, old)
            os.replace(tmp, final)
            with open(os.path.join(self.root, "latest.tmp"), "w") as f:
                f.write(os.path.basename(final))
            os.replace(os.path.join(self.root, "latest.tmp"), os.path.join(self.root, "latest"))
            if old is not None:
                shutil.rmtree(old, ignore_errors=True)
            self._prune(os.path.basename(final))
        self.saved.append(step)
        if dist.is_initialized():
            dist.barrier()

    def _prune(self, current: str) -> None:
        """Keep ``current`` (what ``latest`` now names) and the ``keep - 1`` newest steps before it.  A
        run resumed from an older step re-saves lower step numbers than the directories the abandoned
        run left behind: those (numbered above ``current``) are that run's future, not this one's past,
        and are deleted — kept, they would crowd this run's own checkpoints out of ``keep`` and be what
        ``latest_checkpoint``'s fallback picks if ``latest`` ever names an incomplete directory
        (ADVICE r5).  ``current`` itself is never counted by its number (keep = 1 would delete it)."""
        if self.keep <= 0:
            return
        cur = int(current[5:])
        # numeric order: the zero padding stops sorting lexicographically past step 999999
        steps = sorted((d for d in os.listdir(self.root) if d.startswith("step_") and d[5:].isascii() and d[5:].isdigit() and d != current),
                       key=lambda d: int(d[5:]))
        for d in steps:
            if int(d[5:]) > cur:  # the abandoned run's (complete or not)
                shutil.rmtree(os.path.join(self.root, d), ignore_errors=True)
        older = [d for d in steps if int(d[5:]) < cur and os.path.exists(os.path.join(self.root, d, "meta.json"))]
        for d in older[:max(0, len(older) - (self.keep - 1))]:
            shutil.rmtree(os.path.join(self.root, d), ignore_errors=True)

    def has(self, step: int) -> bool:
        """``step`` is committed or being written."""
        return step in self.saved or (self._pending is not None and self._pending[0] == step)

    def close(self) -> None:
        """Commit the last save (call on every rank before the process group goes away)."""
        self._commit()


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def read_ranges(ckpt_dir: str, ranges: Sequence[Tuple[int, int]], keys=("master", "m", "v")) -> Dict[str, torch.Tensor]:
    """``keys`` over the flat ``ranges`` (concatenated in order), gathered from whichever saved
    rank files hold them — independent of the world size and ZeRO-1 setting they were written at."""
    total = sum(e - s for s, e in ranges)
    out: Dict[str, torch.Tensor] = {}
    filled = 0
    files = sorted(f for f in os.listdir(ckpt_dir) if f.startswith("state_rank") and f.endswith(".safetensors"))
    for fn in files:
        with safe_open(os.path.join(ckpt_dir, fn), framework="pt") as f:
            saved = f.get_tensor("shards").tolist()
            slices = {k: f.get_slice(k) for k in keys}
            for k in keys:
                if k not in out:
                    out[k] = torch.empty(total, dtype=_ST_NAMES[slices[k].get_dtype()])
            off = 0
            for s, e in saved:
                o = 0
                for ws, we in ranges:
                    lo, hi = max(s, ws), min(e, we)
                    if lo < hi:
                        for k in keys:
                            out[k][o + lo - ws:o + hi - ws] = slices[k][off + lo - s:off + hi - s]
                        filled += hi - lo
                    o += we - ws
                off += e - s
    if filled != total or len(out) != len(keys):
        raise ValueError(f"{ckpt_dir}: saved ranges cover {filled} of the {total} elements requested")
    return out


def read_optimizer_ranges(ckpt_dir: str, ranges: Sequence[Tuple[int, int]]) -> Dict[str, torch.Tensor]:
    return read_ranges(ckpt_dir, ranges, ("master", "m", "v"))


def load_checkpoint(path: str, model, opt=None, gen: Optional[torch.Generator] = None) -> Dict[str, object]:
    """Restore weights (and optimizer state / data RNG) from ``path`` — a step directory or a
    checkpoint root (its ``latest``).  Returns the checkpoint's meta (``step`` = steps done)."""
    d = path if os.path.exists(os.path.join(path, "meta.json")) else latest_checkpoint(path)
    if d is None:
        raise FileNotFoundError(f"no committed checkpoint under {path}")
    with open(os.path.join(d, "meta.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{d}: checkpoint format {meta.get('format')} (expected {FORMAT})")
    flat = model.flat
    if meta["numel"] != flat.numel or meta["layout"] != _layout(flat):
        raise ValueError(f"{d}: flat parameter layout does not match this model ({meta['model']!r})")
    w = read_ranges(d, [(0, flat.numel)], ("flat",))["flat"]
    with torch.no_grad():
        flat.data.copy_(w.to(flat.data.dtype), non_blocking=False)
        if hasattr(flat, "invalidate_t"):
            flat.invalidate_t()  # persistent W^T is re-made from the restored weights
    if opt is not None:
        st = read_optimizer_ranges(d, opt.shards)
        dev = opt.master.device
        with torch.no_grad():
            opt.master.copy_(st["master"].to(dev))
            opt.m.copy_(st["m"].to(dev))
            opt.v.copy_(st["v"].to(dev))
        opt.t = int(meta["adam_t"])
    if gen is not None:
        rank, _ = _rank_world()
        p = os.path.join(d, f"rng_rank{rank}.safetensors")
        if os.path.exists(p):  # a rank that did not exist at save time keeps its fresh seed
            with safe_open(p, framework="pt") as f:
                gen.set_state(f.get_tensor("rng"))
    meta["path"] = d
    return meta
