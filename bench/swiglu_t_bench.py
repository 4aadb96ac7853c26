#!/usr/bin/env python3
"""SwiGLU backward at the Llama-3-8B shape: plain kernel + separate transpose vs the fused
transposed-output kernel (swiglu_bwd_t).  python bench/swiglu_t_bench.py [--tokens 16384]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--ffn", type=int, default=14336)
    a = ap.parse_args()
    T, F = a.tokens, a.ffn
    hip = fused.hip()
    gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    dh = torch.randn(T, F, device="cuda", dtype=torch.bfloat16)
    dgu = hip.swiglu_bwd(dh, gu)
    out = {
        "T": T, "F": F,
        "swiglu_bwd_ms": timeit(lambda: hip.swiglu_bwd(dh, gu)),
        "transpose_dgu_ms": timeit(lambda: hip.transpose_bf16(dgu)),
        "swiglu_bwd_t_ms": timeit(lambda: hip.swiglu_bwd_t(dh, gu)),
    }
    for name, (r, c) in {"x": (T, 4096), "ffn": (T, F), "gu": (T, 2 * F), "wqkv": (T, 6144)}.items():
        x = torch.randn(r, c, device="cuda", dtype=torch.bfloat16)
        ms = timeit(lambda: hip.transpose_bf16(x))
        out[f"transpose_{name}_ms"] = ms
        out[f"transpose_{name}_tbps"] = 2 * r * c * 2 / 1e9 / ms
        del x
    gb = (3 * T * F * 2 + 2 * T * F * 2) / 1e9  # read gu + dh, write dgu
    out["swiglu_bwd_tbps"] = gb / out["swiglu_bwd_ms"]
    out["swiglu_bwd_t_tbps"] = (gb + 2 * T * F * 2 / 1e9) / out["swiglu_bwd_t_ms"]
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out.items()}))


if __name__ == "__main__":
    main()
