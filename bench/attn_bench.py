#!/usr/bin/env python3
"""HIP MFMA flash attention vs torch SDPA (ROCm library kernels) at the Llama-3-8B training shape.

    python bench/attn_bench.py [--b 2 --s 4096 --h 32 --hkv 8 --iters 10]

Random gaussian bf16 inputs (guide rule 25: never zeros).  FLOPs counted as causal:
fwd 2 * 2 * B*H*S*S*D / 2, bwd 2.5x fwd.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=2)
    ap.add_argument("--s", type=int, default=4096)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ab", type=int, default=0,
                    help="interleaved A/B of the backward variants: N rounds, one call of each per round, "
                         "event-timed, medians (clock drift hits every variant alike)")
    a = ap.parse_args()
    B, S, H, Hkv, Dh = a.b, a.s, a.h, a.hkv, 128
    q = torch.randn(B, H, S, Dh, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, Dh, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, S, Dh, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(B, S, H, Dh, device="cuda", dtype=torch.bfloat16)
    fwd_flops = 2 * 2 * B * H * S * S * Dh / 2
    res = {"shape": {"B": B, "S": S, "H": H, "Hkv": Hkv, "D": Dh}}
    hip = fused.hip()
    o, lse = hip.attn_fwd(q, k, v, Dh ** -0.5)
    t = timeit(lambda: hip.attn_fwd(q, k, v, Dh ** -0.5), a.iters)
    res["hip_fwd_ms"] = t * 1e3
    res["hip_fwd_tflops"] = fwd_flops / t / 1e12
    t = timeit(lambda: hip.attn_bwd(do, q, k, v, o, lse, Dh ** -0.5), a.iters)
    res["hip_bwd_ms"] = t * 1e3
    res["hip_bwd_tflops"] = 2.5 * fwd_flops / t / 1e12
    if a.ab:
        # interleaved A/B of the backward variants the extension exports (one since round 5: the A/B
        # records of the retired ones are profiles/r05_attn7)
        variants = {"default": lambda: hip.attn_bwd(do, q, k, v, o, lse, Dh ** -0.5)}
        for n in sorted(dir(hip)):
            if n.startswith("attn_bwd_"):
                variants[n] = (lambda fn: lambda: fn(do, q, k, v, o, lse, Dh ** -0.5))(getattr(hip, n))
        times = {n: [] for n in variants}
        for fn in variants.values():
            fn()
        for _ in range(a.ab):
            for n, fn in variants.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                times[n].append((e0, e1))
        torch.cuda.synchronize()
        res["ab_median_ms"] = {n: sorted(x.elapsed_time(y) for x, y in ts)[len(ts) // 2] for n, ts in times.items()}
        ref = variants["default"]()
        res["ab_rel_vs_default"] = {n: [float(((x.float() - y.float()).norm() / y.float().norm()).item()) for x, y in zip(fn(), ref)]
                                    for n, fn in variants.items()}
        # forward variants (attn_fwdv_*), interleaved against attn_fwd the same way
        fvars = {"fwd": lambda: hip.attn_fwd(q, k, v, Dh ** -0.5)}
        for n in sorted(dir(hip)):
            if n.startswith("attn_fwdv_"):
                fvars[n] = (lambda fn: lambda: fn(q, k, v, Dh ** -0.5))(getattr(hip, n))
        if len(fvars) > 1:
            ft = {n: [] for n in fvars}
            for fn in fvars.values():
                fn()
            for _ in range(a.ab):
                for n, fn in fvars.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    ft[n].append((e0, e1))
            torch.cuda.synchronize()
            res["ab_fwd_median_ms"] = {n: sorted(x.elapsed_time(y) for x, y in ts)[len(ts) // 2] for n, ts in ft.items()}
            fref = fvars["fwd"]()
            res["ab_fwd_rel"] = {n: [float(((x.float() - y.float()).norm() / y.float().norm()).item()) for x, y in zip(fn(), fref)]
                                 for n, fn in fvars.items()}
    try:
        t = timeit(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True), a.iters)
        res["sdpa_fwd_ms"] = t * 1e3
        res["sdpa_fwd_tflops"] = fwd_flops / t / 1e12
        qq, kk, vv = (x.clone().requires_grad_(True) for x in (q, k, v))
        out = F.scaled_dot_product_attention(qq, kk, vv, is_causal=True, enable_gqa=True)
        g = do.transpose(1, 2).contiguous()
        t = timeit(lambda: torch.autograd.grad(out, (qq, kk, vv), g, retain_graph=True), a.iters)
        res["sdpa_bwd_ms"] = t * 1e3
        res["sdpa_bwd_tflops"] = 2.5 * fwd_flops / t / 1e12
    except Exception as e:  # pragma: no cover
        res["sdpa_error"] = str(e)[:300]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
