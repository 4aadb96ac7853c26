#!/usr/bin/env python3
"""Library GEMMs of the Llama-3-8B step with hot vs cold operands (MI355X's 256 MB Infinity Cache).

    python bench/gemm_cold_bench.py [--tokens 16384] [--reps 8] [--table PATH] [--tune-out PATH --rotating-mb 1024]

In the training step the forward projections ran 20-40 % slower than the same shapes in the TunableOp
table (profiles/r03_llama2): there the weight comes cold from HBM, while the tuning loop (and the
backward, whose W^T / x^T were just written by the transpose kernel) finds its operands in the
Infinity Cache.  For each forward shape ``y = x W^T`` this times, interleaved, event-timed, medians:

* ``hot``      the GEMM right after the same GEMM (operands resident);
* ``cold_w``   as in the step: a 1 GiB write flushes the Infinity Cache, x is touched (as its producer
  would leave it), W comes from HBM;
* ``prefetch`` the same, with a streaming read of W (a reduction) right before the GEMM: is a cheap
  prefetch worth it?  Reported as GEMM-only and prefetch+GEMM times.

``--tune-out``: first re-tune these shapes with TunableOp's rotating buffer (``--rotating-mb``, so every
tuning call sees cold operands; TunableOp writes the table at exit) into a new table, then time with that table.
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.models.gemm_tuning import DEFAULT_TABLE, setup_gemm_tuning  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--table", default=DEFAULT_TABLE)
    ap.add_argument("--tune-out", default="")
    ap.add_argument("--rotating-mb", type=int, default=4096)
    ap.add_argument("--shapes", default="wqkv,wo,w13,w2")
    a = ap.parse_args()
    T, D, FF = a.tokens, 4096, 14336
    shapes = {"wqkv": (6144, D), "wo": (D, D), "w13": (2 * FF, D), "w2": (D, FF), "lm_head": (128256, D)}
    names = [s for s in a.shapes.split(",") if s]
    import torch.cuda.tunable as tunable

    if a.tune_out:
        tunable.enable(True)
        tunable.tuning_enable(True)
        tunable.set_rotating_buffer_size(a.rotating_mb)
        tunable.set_max_tuning_duration(10)
        tunable.set_max_tuning_iterations(10)
        tunable.set_filename(a.tune_out, False)
        for n in names:
            N, K = shapes[n]
            x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            torch.mm(x, w.t())
            torch.cuda.synchronize()
            print(f"tuned {n}", flush=True)
            del x, w
        tunable.tuning_enable(False)
        mode = "tuned-rotating"
        table = a.tune_out
    else:
        mode = setup_gemm_tuning("use", a.table)
        table = a.table
    flush = torch.empty(1 << 29, device="cuda", dtype=torch.float16)  # 1 GiB: more than the Infinity Cache
    out = {"tokens": T, "mode": mode, "table": os.path.basename(table), "rotating_mb": a.rotating_mb if a.tune_out else None,
           "shapes": []}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for n in names:
        N, K = shapes[n]
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        y = F.linear(x, w)
        torch.cuda.synchronize()
        t = {"hot": [], "cold_w": [], "prefetch_gemm": [], "prefetch_total": []}
        for _ in range(a.reps):
            # hot: the same GEMM twice, the second timed
            torch.mm(x, w.t(), out=y)
            ev[0].record()
            torch.mm(x, w.t(), out=y)
            ev[1].record()
            # as in the step: the Infinity Cache flushed, x just touched (its producer), W cold
            flush.fill_(1.0)
            x.sum()
            ev[2].record()
            torch.mm(x, w.t(), out=y)
            ev[3].record()
            torch.cuda.synchronize()
            t["hot"].append(ev[0].elapsed_time(ev[1]))
            t["cold_w"].append(ev[2].elapsed_time(ev[3]))
            # the same, with a streaming read of W (a reduction) right before the GEMM
            flush.fill_(2.0)
            x.sum()
            ev[0].record()
            w.sum()
            ev[1].record()
            torch.mm(x, w.t(), out=y)
            ev[2].record()
            torch.cuda.synchronize()
            t["prefetch_gemm"].append(ev[1].elapsed_time(ev[2]))
            t["prefetch_total"].append(ev[0].elapsed_time(ev[2]))
        flop = 2.0 * T * N * K
        row = {"name": n, "M_N_K": [T, N, K], "w_mb": round(N * K * 2 / 2**20, 1)}
        for k, v in t.items():
            ms = statistics.median(v)
            row[f"{k}_ms"] = round(ms, 4)
            if k != "prefetch_total":
                row[f"{k}_tflops"] = round(flop / (ms / 1e3) / 1e12, 1)
        out["shapes"].append(row)
        print(json.dumps(row), flush=True)
        del x, w, y
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
