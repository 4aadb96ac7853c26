#!/usr/bin/env python3
"""K3 HBM self-copy probe: variant sweep on one MI355X (where does the copy kernel sit against the
guide's 6.29 TB/s float4-copy measurement?).

    python bench/copy_sweep.py [--sizes 256M,2G] [--out gpurun_out/copy_sweep.json]

Rows: kind (lds = LDS-DMA staged, reg = register staged, chunk/chunk4 = one contiguous slice per
workgroup with 8/4 loads in flight, sdma = hipMemcpyAsync), non-temporal stores,
workgroups per CU; GB/s is the copy rate (bytes copied / s), HBM traffic is twice that."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from gpu_topology_on_k8s_amd.ops import probe

    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256M,2G")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--kinds", default="lds,reg,chunk,chunk4,sdma")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    mult = {"M": 1 << 20, "G": 1 << 30}
    rows = []
    for sz in a.sizes.split(","):
        nbytes = int(float(sz[:-1]) * mult[sz[-1]])
        for kind in a.kinds.split(","):
            for nt in ((False, True) if kind in ("lds", "reg") else (True,) if kind.startswith("chunk") else (False,)):
                for bpc in ((2, 4, 8, 16) if kind != "sdma" else (8,)):
                    r = probe.copy_bw(0, 0, nbytes, iters=a.iters, warmup_iters=2, kind=kind, nontemporal=nt, blocks_per_cu=bpc)
                    row = {"bytes": nbytes, "kind": kind, "nt": nt, "blocks_per_cu": bpc, "copy_gbps": round(r["gbps"], 1),
                           "hbm_tbps": round(2 * r["gbps"] / 1e3, 3), "ok": bool(r["ok"])}
                    print(json.dumps(row), flush=True)
                    rows.append(row)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
