#!/usr/bin/env python3
"""Does the relative placement of source and destination in HBM change device-to-device copy speed?

The k = 1 headline is RCCL's one-rank all-reduce, which RCCL runs as a runtime device-to-device
copy of the send buffer into the receive buffer.  HBM3E interleaves addresses over channels and
banks, so a read stream and a write stream whose addresses differ by a large power of two can land
on the same channels in lock step.  This script times ``dst.copy_(src)`` (hipMemcpyAsync D2D, the
runtime blit) for two separate allocations and for one allocation carved at several offsets.

    python bench/copy_layout.py --mib 2048 --iters 20
"""
from __future__ import annotations

import argparse
import json


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--mib", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sweep", action="store_true", help="dense sweep of dst-src gaps (4 KiB .. 64 MiB, both orders)")
    a = ap.parse_args()
    import torch

    n = a.mib << 20
    torch.cuda.set_device(0)

    def timed(src, dst):
        dst.copy_(src)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            dst.copy_(src)
        e1.record()
        torch.cuda.synchronize()
        return n * a.iters / (e0.elapsed_time(e1) / 1e3) / 1e9

    rows = []
    src, dst = torch.ones(n, dtype=torch.uint8, device="cuda"), torch.empty(n, dtype=torch.uint8, device="cuda")
    rows.append({"layout": "separate", "dst_minus_src": dst.data_ptr() - src.data_ptr(), "algbw_gbps": round(timed(src, dst), 1)})
    del src, dst
    torch.cuda.empty_cache()
    pad = 64 << 20
    big = torch.empty(2 * n + pad, dtype=torch.uint8, device="cuda")
    big[:n].fill_(1)
    offs = [0, 256, 4096, 65536, 1 << 20, (1 << 20) + 4096, 2 << 20, (2 << 20) + 256 * 1024, 3 << 20, 16 << 20,
            (16 << 20) + 8192, 32 << 20]
    if a.sweep:
        import random

        rng = random.Random(1)
        offs = sorted(set([k << 12 for k in range(0, 64)] + [k << 16 for k in range(0, 64)] + [k << 20 for k in range(0, 64)]
                          + [rng.randrange(0, 64 << 20) & ~4095 for _ in range(64)]))
    for off in offs:
        src, dst = big[:n], big[n + off:2 * n + off]
        rows.append({"layout": "one-alloc", "gap": off, "dst_minus_src": dst.data_ptr() - src.data_ptr(),
                     "algbw_gbps": round(timed(src, dst), 1)})
    for r in rows:
        print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
