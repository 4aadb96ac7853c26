#!/usr/bin/env python3
"""Library GEMM (hipBLASLt via torch) throughput at the Llama-3-8B training shapes.

    python bench/gemm_bench.py [--tokens 16384 --iters 10]

For every projection (wqkv, wo, w13, w2, lm_head) the three GEMMs of a training step are timed:
fwd ``y = x W^T``, dgrad ``dx = dy W`` and wgrad ``dW = dy^T x``.  Random gaussian bf16 operands.
This is the evidence for the step breakdown in README (GEMMs ~64% of the Llama step) and the
yard-stick any hand-written MFMA GEMM has to beat.
"""
import argparse
import json
import time

import torch


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    T, D, F, V = a.tokens, 4096, 14336, 128256
    shapes = {"wqkv": (6144, D), "wo": (D, D), "w13": (2 * F, D), "w2": (D, F), "lm_head": (V, D)}
    out = {"tokens": T, "gemms": []}
    total_flop, total_s = 0.0, 0.0
    for name, (N, K) in shapes.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * T * N * K
        for kind, fn in (("fwd", lambda: x @ w.t()), ("dgrad", lambda: dy @ w), ("wgrad", lambda: dy.t() @ x)):
            t = timeit(fn, a.iters)
            out["gemms"].append({"name": name, "kind": kind, "M_N_K": [T, N, K] if kind != "wgrad" else [N, K, T],
                                 "ms": round(t * 1e3, 3), "tflops": round(flop / t / 1e12, 1)})
            total_flop += flop
            total_s += t
        del x, w, dy
        torch.cuda.empty_cache()
    out["aggregate_tflops"] = round(total_flop / total_s / 1e12, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
