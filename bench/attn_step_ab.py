#!/usr/bin/env python3
"""Interleaved A/B of the Llama-3-8B training step (BASELINE config 5, one GPU) with the attention
backward of another build of the ``_fused`` extension against this tree's.

    python bench/attn_step_ab.py --so scratch/r04/_fused.cpython-310-x86_64-linux-gnu.so [--rounds 4 --steps 3]

The other build (e.g. the round-4 tree, ``git worktree add /tmp/r04 <rev>`` + ``_native.build``) is
loaded as a second extension module; only ``attn_bwd`` is switched, every other kernel is this tree's.
One model, one optimizer, one process: the arms alternate every ``--steps`` steps, so clock and
thermal drift hit both alike.  A step is the training step of models/train.py at world 1: forward,
backward, fused AdamW (with W^T).  Prints one JSON line: per-arm ms/step of every round and medians.
"""
import argparse
import importlib.machinery
import importlib.util
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.models import FlatAdamW, Llama, LlamaConfig  # noqa: E402
from gpu_topology_on_k8s_amd.models.gemm_tuning import setup_gemm_tuning  # noqa: E402
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def load_other(path: str):
    loader = importlib.machinery.ExtensionFileLoader("_fused", os.path.abspath(path))
    spec = importlib.util.spec_from_loader("_fused", loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


class Switch:
    """``fused.hip()`` stand-in: this tree's extension, with the ``swap`` entry points (default
    ``attn_bwd``) from ``other`` when ``use_other``."""

    def __init__(self, cur, other, swap=("attn_bwd",)):
        self.cur, self.other, self.use_other, self.swap = cur, other, False, tuple(swap)

    def __getattr__(self, name):
        if name in self.swap and self.use_other:
            return getattr(self.other, name)
        return getattr(self.cur, name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", required=True)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--swap", default="attn_bwd", help="comma-separated entry points taken from the other build")
    a = ap.parse_args()
    sw = Switch(fused.hip(), load_other(a.so), swap=[x for x in a.swap.split(",") if x])
    fused.hip = lambda: sw  # every call site goes through fused.hip()
    setup_gemm_tuning("auto", None, 0)
    cfg = LlamaConfig.named(a.model)
    model = Llama(cfg, device="cuda", seed=0)
    opt = FlatAdamW(model.flat, lr=3e-4)
    g = torch.Generator().manual_seed(1234)
    toks = [torch.randint(0, cfg.vocab, (a.batch, a.seq + 1), generator=g).cuda() for _ in range(4)]

    def step(i):
        t = toks[i % len(toks)]
        model.flat.zero_grad()
        loss = model(t[:, :-1], t[:, 1:])
        loss.backward()
        opt.step()
        return loss

    for arm in (False, True):  # warm both arms (TunableOp lookups, allocator, first launches)
        sw.use_other = arm
        for i in range(2):
            step(i)
    torch.cuda.synchronize()
    times = {"this": [], "other": []}
    n = 0
    for _ in range(a.rounds):
        for arm in (False, True):
            sw.use_other = arm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(n)
                n += 1
            torch.cuda.synchronize()
            times["other" if arm else "this"].append((time.perf_counter() - t0) / a.steps * 1e3)
    med = {k: statistics.median(v) for k, v in times.items()}
    print(json.dumps({"model": a.model, "batch": a.batch, "seq": a.seq, "other_so": a.so, "swap": sw.swap, "ms_per_step": times,
                      "median_ms": med, "delta_pct": 100.0 * (med["this"] / med["other"] - 1.0),
                      "tokens_per_s_this": a.batch * a.seq / med["this"] * 1e3}), flush=True)


if __name__ == "__main__":
    main()
