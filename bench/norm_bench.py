"""Fused residual add + RMSNorm vs add + RMSNorm at the Llama-3-8B shape (T = 16384, D = 4096, bf16).

    python bench/norm_bench.py

Buffers rotate over 6 sets (≈2.4 GB) so each call streams from HBM, not the 256 MB MALL.
Reports µs per call and the HBM rate implied by the minimum bytes each variant must move.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_topology_on_k8s_amd.ops import fused


def timeit(fn, n=50):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(n):
        fn(i)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    hip = fused.hip()
    T, D, K = 16384, 4096, 6
    g = torch.Generator(device="cuda").manual_seed(0)
    mk = lambda: torch.randn(T, D, device="cuda", dtype=torch.bfloat16, generator=g)  # noqa: E731
    xs, rs, dys, dhs = [mk() for _ in range(K)], [mk() for _ in range(K)], [mk() for _ in range(K)], [mk() for _ in range(K)]
    w = (torch.rand(D, device="cuda") + 0.5).to(torch.bfloat16)
    hs, rstds = [], []
    for i in range(K):
        h, _, rstd = hip.add_rmsnorm_fwd(xs[i], rs[i], w, 1e-5)
        hs.append(h)
        rstds.append(rstd)
    P = T * D * 2
    rows = {
        "fused_fwd": (timeit(lambda i: hip.add_rmsnorm_fwd(xs[i % K], rs[i % K], w, 1e-5)), 4 * P),
        "unfused_fwd": (timeit(lambda i: hip.rmsnorm_fwd(xs[i % K] + rs[i % K], w, 1e-5)), 5 * P),
        "fused_bwd": (timeit(lambda i: hip.add_rmsnorm_bwd(dys[i % K], hs[i % K], w, rstds[i % K], dhs[i % K])), 4 * P),
        "unfused_bwd": (timeit(lambda i: hip.rmsnorm_bwd(dys[i % K], hs[i % K], w, rstds[i % K])[0] + dhs[i % K]), 6 * P),
    }
    for k, (us, nbytes) in rows.items():
        print(json.dumps({"case": k, "T": T, "D": D, "us": round(us, 1), "min_bytes": nbytes,
                          "tbps": round(nbytes / (us * 1e-6) / 1e12, 2)}))


if __name__ == "__main__":
    main()
