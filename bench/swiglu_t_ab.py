#!/usr/bin/env python3
"""Interleaved A/B of the SwiGLU backward-with-transpose kernels at the Llama-3-8B shape
(T 16384, F 14336): 64 x 64 tiles (swiglu_bwd_t) vs 64 x 128 (swiglu_bwd_t128); event-timed medians."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def main():
    T, F = 16384, 14336
    gu = torch.randn(T, 2 * F, device="cuda", dtype=torch.bfloat16)
    dh = torch.randn(T, F, device="cuda", dtype=torch.bfloat16)
    hip = fused.hip()
    fns = {"t64": hip.swiglu_bwd_t, "t128": hip.swiglu_bwd_t128}
    for f in fns.values():
        f(dh, gu)
    times = {n: [] for n in fns}
    for _ in range(30):
        for n, f in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f(dh, gu)
            e1.record()
            times[n].append((e0, e1))
    torch.cuda.synchronize()
    nbytes = (T * F + 2 * T * 2 * F) * 2 + T * 2 * F * 2  # dh + gu in, dgu + dgu^T out
    out = {}
    for n, ts in times.items():
        ms = sorted(a.elapsed_time(b) for a, b in ts)[len(ts) // 2]
        out[n] = {"ms": round(ms, 4), "tb_s": round(nbytes / ms / 1e9, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
