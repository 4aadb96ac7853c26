#!/usr/bin/env python3
"""Which operand layout makes the library GEMMs of a Llama-3-8B training step fastest?

    python bench/gemm_layout_bench.py [--tokens 16384 --iters 10 --tune]

For every projection (y = x W^T) the backward GEMMs are timed in the layout autograd hands them to
hipBLASLt and in the "NT" layout of the forward GEMM (both operands contiguous along the reduction
dimension), together with the transposes that layout needs:

  dgrad  dx = dy W        (NN)   vs  dx = dy (W^T)^T     with W^T materialised once per step
  wgrad  dW = dy^T x      (TN)   vs  dW = (dy^T)(x^T)^T  with dy^T and x^T materialised per layer

``--tune`` lets TunableOp time every hipBLASLt/rocBLAS solution for each shape first (fresh table
under gpurun_out/), so both layouts are compared at their best kernels.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.ops import fused


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
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--only", default="", help="comma list of projections (default: all)")
    a = ap.parse_args()
    if a.tune:
        import torch.cuda.tunable as tunable

        os.makedirs("gpurun_out", exist_ok=True)
        tunable.enable(True)
        tunable.tuning_enable(True)
        tunable.set_max_tuning_duration(10)
        tunable.set_max_tuning_iterations(10)
        tunable.set_filename("gpurun_out/tunableop_layout.csv", False)
    T, D, F, V = a.tokens, 4096, 14336, 128256
    shapes = {"wqkv": (6144, D), "wo": (D, D), "w13": (2 * F, D), "w2": (D, F), "lm_head": (V, D)}
    rows = []
    for name, (N, K) in shapes.items():
        if a.only and name not in a.only.split(","):
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g)
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16, generator=g)
        wT, dyT, xT = w.t().contiguous(), dy.t().contiguous(), x.t().contiguous()
        flop = 2.0 * T * N * K
        # numerics: the NT forms compute the same products
        ref_dx, ref_dw = (dy @ w).float(), (dy.t() @ x).float()
        err_dx = ((dy @ wT.t()).float() - ref_dx).abs().max().item() / ref_dx.abs().max().item()
        err_dw = ((dyT @ xT.t()).float() - ref_dw).abs().max().item() / ref_dw.abs().max().item()
        del ref_dx, ref_dw
        r = {"name": name, "N": N, "K": K, "T": T}
        for kind, fn in (("fwd_nt", lambda: x @ w.t()),
                         ("dgrad_nn", lambda: dy @ w), ("dgrad_nt", lambda: dy @ wT.t()),
                         ("wgrad_tn", lambda: dy.t() @ x), ("wgrad_nt", lambda: dyT @ xT.t()),
                         ("transpose_w", lambda: w.t().contiguous()), ("transpose_dy", lambda: dy.t().contiguous()),
                         ("transpose_x", lambda: x.t().contiguous()),
                         ("hip_transpose_w", lambda: fused.transpose(w)), ("hip_transpose_dy", lambda: fused.transpose(dy)),
                         ("hip_transpose_x", lambda: fused.transpose(x))):
            t = timeit(fn, a.iters)
            r[kind + "_ms"] = round(t * 1e3, 4)
            if "transpose" in kind:
                r[kind + "_tbps"] = round(2 * {"w": w, "dy": dy, "x": x}[kind.rsplit("_", 1)[1]].numel() * 2 / t / 1e12, 2)
            else:
                r[kind + "_tflops"] = round(flop / t / 1e12, 1)
        r["rel_err_dgrad_nt"] = err_dx
        r["rel_err_wgrad_nt"] = err_dw
        r["wgrad_nt_incl_transposes_ms"] = round(r["wgrad_nt_ms"] + r["hip_transpose_dy_ms"] + r["hip_transpose_x_ms"], 4)
        r["dgrad_nt_incl_transpose_ms"] = round(r["dgrad_nt_ms"] + r["hip_transpose_w_ms"], 4)
        rows.append(r)
        print(json.dumps(r), flush=True)
        del x, w, dy, wT, dyT, xT
        torch.cuda.empty_cache()
    print(json.dumps({"summary": True, "tuned": a.tune, "rows": rows}))


if __name__ == "__main__":
    main()
