#!/usr/bin/env python3
"""Placement core on a CPX node (64 XCPs in 8 packages, three XCPs busy): search nodes, time, exactness
and objective per request size.  ``python bench/cpx_placement_bench.py`` -> one JSON line per k."""
import json
import os
import sys
import time

sys.path.insert(0, os.environ.get("GTK_REPO", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gpu_topology_on_k8s_amd.placement import select  # noqa: E402
from gpu_topology_on_k8s_amd.topology import fixtures as fx  # noqa: E402


def main():
    t = fx.f8_mi355x_cpx(link_gbps=76.5, noise=0.05, seed=2)
    for k in (2, 4, 8, 12, 16, 20, 24, 32, 40, 48, 56):
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            pl = select(t, k, used=[0, 9, 18])
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        print(json.dumps({"k": k, "ms": round(best * 1e3, 1), "nodes": int(pl.terms["search_nodes"]), "exact": pl.exact,
                          "objective": round(pl.objective, 4), "packages": len({t.gpus[i].physical for i in pl.ids})}), flush=True)


if __name__ == "__main__":
    main()
