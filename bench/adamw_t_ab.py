#!/usr/bin/env python3
"""AdamW-T tile kernel look-ahead A/B at the Llama-3-8B parameter layout: 1, 2 or 4 eight-row passes'
loads issued before their stores (csrc/ops/adamw_t.hip kAhead), interleaved, event-timed medians."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.models import FlatAdamW, Llama, LlamaConfig  # noqa: E402
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def main():
    m = Llama(LlamaConfig.llama3_8b(), device="cuda", seed=0)
    opt = FlatAdamW(m.flat, lr=3e-4)
    m.flat.grad.normal_(0, 1e-3)
    mats, tiles, ranges, maxr = m.flat.adamw_plan()
    hip = fused.hip()
    hp = torch.tensor([3e-4, 0.9, 0.95, 1e-8, 0.1, 1.0, 0.1, 0.05], device="cuda")

    def run(a):
        hip.adamw_step_t(opt.master, opt.m, opt.v, m.flat.grad, m.flat.data, m.flat.data_t, hp, mats, tiles, ranges, maxr,
                         None, None, a)

    for a in (1, 2, 4):
        run(a)
    ev = {a: [] for a in (1, 2, 4)}
    for _ in range(8):
        for a in (1, 2, 4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(a)
            e1.record()
            ev[a].append((e0, e1))
    torch.cuda.synchronize()
    print(json.dumps({f"ahead{a}_ms": round(sorted(x.elapsed_time(y) for x, y in v)[len(v) // 2], 3) for a, v in ev.items()}),
          flush=True)


if __name__ == "__main__":
    main()
