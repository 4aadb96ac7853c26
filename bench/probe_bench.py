#!/usr/bin/env python3
"""Probe-kernel sweep: staging kind x store flavour x size, HBM self-copy and (if >1 GPU) p2p.

    python bench/probe_bench.py [--out gpurun_out/probe.json] [--sizes 64,256,1024] [--iters 10]

Used under rocprofv3 to document the gfx950 tiling of the K1-K4 kernels (profiles/).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_topology_on_k8s_amd.ops import probe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--sizes", default="64,256,1024")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--bpcu", default="8")
    a = ap.parse_args()
    n = probe.device_count()
    res = {"devices": n, "props": probe.device_props(0), "warmup": probe.warmup(0, 100.0), "hbm": [], "p2p": []}
    for mb in [int(x) for x in a.sizes.split(",")]:
        for kind in ("lds", "reg", "sdma"):
            for nt in ((False, True) if kind != "sdma" else (False,)):
                for bpcu in [int(x) for x in a.bpcu.split(",")]:
                    r = probe.copy_bw(0, 0, mb << 20, iters=a.iters, warmup_iters=2, kind=kind, nontemporal=nt, blocks_per_cu=bpcu)
                    r["hbm_traffic_gbps"] = 2 * r["gbps"]
                    res["hbm"].append(r)
                    print(f"hbm {mb:5d} MiB {kind:4s} nt={int(nt)} bpcu={bpcu}: copy {r['gbps']:7.1f} GB/s "
                          f"(HBM r+w {2 * r['gbps']:7.1f}) ok={r['ok']}", flush=True)
    if n > 1:
        for mode in ("read", "write"):
            m = probe.measure_matrix(list(range(n)), 256 << 20, 5, 1, mode=mode)
            res["p2p"].append({"mode": mode, "matrix_gbps": m.tolist()})
            print(mode, m.round(1))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
