#!/usr/bin/env python3
"""Producer-written transposes vs a separate transpose pass, at the Llama-3-8B b4 x 4096 shapes
(event-timed medians, interleaved):
  swiglu forward   T 16384, F 14336: swiglu_fwd (+ transpose) vs swiglu_fwd_t (64x64) vs swiglu_fwd_t128
  xent backward    T 16384, V 128256: xent_bwd_inplace (+ transpose) vs xent_bwd_t
  RoPE backward    B 4, H 32, Hkv 8, S 4096: rope_split_bwd (+ transpose) vs rope_split_bwd_t
  attention fwd    B 4, H 32, Hkv 8, S 4096: attn_fwd (+ transpose of O) vs attn_fwd_t
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def timed(fns, reps=20):
    for f in fns.values():
        f()
    ev = {n: [] for n in fns}
    for _ in range(reps):
        for n, f in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            ev[n].append((a, b))
    torch.cuda.synchronize()
    return {n: round(sorted(a.elapsed_time(b) for a, b in v)[len(v) // 2], 4) for n, v in ev.items()}


def main():
    hip = fused.hip()
    out = {}
    T, F = 16384, 14336
    gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    out["swiglu_fwd_ms"] = timed({
        "fwd": lambda: hip.swiglu_fwd(gu),
        "fwd+transpose": lambda: hip.transpose_bf16(hip.swiglu_fwd(gu)),
        "fwd_t64": lambda: hip.swiglu_fwd_t(gu),
        "fwd_t128": lambda: hip.swiglu_fwd_t128(gu),
    })
    del gu
    torch.cuda.empty_cache()
    V = 128256
    logits = (torch.randn(T, V, device="cuda") * 2).to(torch.bfloat16)
    labels = torch.randint(0, V, (T,), device="cuda")
    _, lse = hip.xent_fwd(logits, labels, -100)
    sc = torch.tensor([1.0 / T], device="cuda")
    work = logits.clone()
    out["xent_bwd_ms"] = timed({
        "inplace": lambda: hip.xent_bwd_inplace(work, labels, lse, sc, -100),
        "inplace+transpose": lambda: (hip.xent_bwd_inplace(work, labels, lse, sc, -100), hip.transpose_bf16(work)),
        "bwd_t": lambda: hip.xent_bwd_t(work, labels, lse, sc, -100),
    }, reps=10)
    del logits, work
    torch.cuda.empty_cache()
    B, H, Hkv, S = 4, 32, 8, 4096
    cos, sin = fused.rope_tables(S, 128, device="cuda")
    dq = torch.randn(B, H, S, 128, device="cuda", dtype=torch.bfloat16)
    dk = torch.randn(B, Hkv, S, 128, device="cuda", dtype=torch.bfloat16)
    dv = torch.randn(B, Hkv, S, 128, device="cuda", dtype=torch.bfloat16)
    out["rope_bwd_ms"] = timed({
        "bwd": lambda: hip.rope_split_bwd(dq, dk, dv, cos, sin, 0),
        "bwd+transpose": lambda: hip.transpose_bf16(hip.rope_split_bwd(dq, dk, dv, cos, sin, 0)),
        "bwd_t": lambda: hip.rope_split_bwd_t(dq, dk, dv, cos, sin, 0),
    })
    del dq, dk, dv
    q = torch.randn(B, H, S, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, S, 128, device="cuda", dtype=torch.bfloat16)
    sc = 128 ** -0.5
    out["attn_fwd_ms"] = timed({
        "fwd": lambda: hip.attn_fwd(q, k, v, sc),
        "fwd+transpose": lambda: hip.transpose_bf16(hip.attn_fwd(q, k, v, sc)[0].view(B * S, H * 128)),
        "fwd_t": lambda: hip.attn_fwd_t(q, k, v, sc),
    })
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
