#!/usr/bin/env python3
"""Input-gradient GEMM from the transposed gradient: is ``dx = dy @ W`` as fast when dy arrives only as
``dy^T`` (hipBLASLt's transposed-A path) as from a row-major ``dy``?

The backward producers (SwiGLU, RoPE, cross-entropy; ``ops/fused.py``) write their gradient in both
layouts: row-major for the input-gradient GEMM, transposed for the NT-layout weight-gradient GEMM.  If
the input-gradient GEMM ran at the same rate from ``dy^T``, each producer could write one layout only
(940 MB less per layer for SwiGLU, 4.2 GB per step for the logits).  Interleaved timing of both forms
for the Llama-3-8B shapes, TunableOp tuning both:

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 python bench/dgrad_layout_bench.py
"""
import json
import statistics

import torch
import torch.nn.functional as F


def timed(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    T = 16384
    shapes = {"w13 (swiglu)": (28672, 4096), "wqkv (rope)": (6144, 4096), "lm_head (xent)": (128256, 4096)}
    out = {}
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (fo, fi) in shapes.items():
        dy = torch.randn(T, fo, device="cuda", dtype=torch.bfloat16, generator=g)
        dy_t = dy.t().contiguous()
        w_t = torch.randn(fi, fo, device="cuda", dtype=torch.bfloat16, generator=g)  # persistent W^T [in, out]
        a = lambda: F.linear(dy, w_t)  # noqa: E731 - production: row-major dy, NT
        b = lambda: F.linear(dy_t.t(), w_t)  # noqa: E731 - from dy^T: transposed A
        for f in (a, b):
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        ta, tb = [], []
        for _ in range(7):
            ta.append(timed(a))
            tb.append(timed(b))
        ref, alt = a(), b()
        out[name] = {"rowmajor_ms": round(statistics.median(ta), 4), "from_transposed_ms": round(statistics.median(tb), 4),
                     "delta_pct": round(100 * (statistics.median(tb) / statistics.median(ta) - 1), 2),
                     "max_abs_diff": float((ref.float() - alt.float()).abs().max()),
                     "tflops_rowmajor": round(2 * T * fo * fi / statistics.median(ta) / 1e9, 1)}
        print(json.dumps({name: out[name]}), flush=True)
        del dy, dy_t, w_t, ref, alt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
