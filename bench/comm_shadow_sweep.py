#!/usr/bin/env python3
"""What 8-GPU data parallelism's gradient all-reduces would cost the Llama-3-8B step, on one GPU
(VERDICT r3 next #4).

    python bench/comm_shadow_sweep.py [--ctas 0,8,16,32,64] [--busbw 350] [--out gpurun_out/x/shadow.jsonl]

For each CTA count N, one training run (models/train.py) whose bucket-ready hooks launch the shadow
of the ring all-reduce an 8-rank job would start there (parallel/dp.py CommShadow): N workgroups copy
the bucket's ring traffic, 2 (k-1)/k of its bytes, paced over ring_bytes / busBW, on a side stream.
N = 0 is the plain step.  ``--zero1`` plays ZeRO-1's reduce-scatter (at the hook) and weight all-gather
(after the optimizer, waited per bucket by the next forward) instead of the all-reduce.  Each line: ms/step, the inflation over N = 0, and the collective time the
shadow represents (which would be fully exposed without overlap).  The DP cap (--comm-ctas) is chosen
from this curve: the smallest N whose collectives still finish inside the backward, at the lowest
inflation (profiles/r04_comm_shadow).
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(ctas, a):
    cmd = [sys.executable, "-m", "gpu_topology_on_k8s_amd.models.train", "--model", a.model, "--batch", str(a.batch),
           "--seq", str(a.seq), "--steps", str(a.steps), "--warmup", str(a.warmup), "--comm-shadow", str(ctas),
           "--comm-shadow-busbw", str(a.busbw), "--comm-shadow-k", str(a.k)] + (["--zero1"] if a.zero1 else [])
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run(cmd, capture_output=True, text=True, cwd=REPO, env=env, timeout=a.timeout)
    if p.returncode != 0:
        raise RuntimeError(f"ctas={ctas}: exit {p.returncode}\n{p.stderr[-2000:]}")
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctas", default="0,8,16,32,64")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--busbw", type=float, default=350.0)
    ap.add_argument("--timeout", type=float, default=600)
    ap.add_argument("--zero1", action="store_true",
                    help="shadow ZeRO-1's traffic instead: each bucket's reduce-scatter at its hook and its weight "
                         "all-gather after the optimizer, (k-1)/k of the bucket each (parallel/dp.py CommShadow)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    base = None
    for n in [int(x) for x in a.ctas.split(",")]:
        r = run(n, a)
        ms = r["ms_per_step"]
        base = ms if n == 0 else base
        sh = r.get("comm_shadow") or {}
        line = {"ctas": n, "ms_per_step": round(ms, 2), "tokens_per_s": round(r["tokens_per_s"], 1),
                "inflation": round(ms / base - 1, 4) if base else None,
                "collective_ms_per_step": round(sh.get("collective_us_per_step", 0) / 1e3, 2),
                "achieved_ms_per_step": round(sh.get("achieved_ms_per_step", 0), 2),
                "exposed_ms_per_step": round(sh.get("exposed_ms_per_step", 0), 2),
                "collectives_per_step": sh.get("collectives_per_step"), "ring_gb_per_step": round(sh.get("ring_bytes_per_step", 0) / 1e9, 2),
                "k": a.k, "busbw_gbps": a.busbw, "model": a.model, "batch": a.batch, "seq": a.seq, "zero1": a.zero1}
        print(json.dumps(line), flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
