"""K3 HBM self-copy variants on one MI355X, far past the Infinity Cache: which copy kernel and
occupancy the probe's HBM reference should use (profiles/r06_prof).

    python bench/hbm_copy_sweep.py [--bytes 1073741824] [--rounds 3]

Prints one JSON line per (kind, non-temporal, blocks per CU), each the median of ``--rounds``
interleaved measurements, and a final line naming the fastest."""
import argparse
import json
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpu_topology_on_k8s_amd.ops import probe  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    arms = [(k, nt, b) for k in ("lds", "reg", "chunk4", "chunk") for nt in (False, True) for b in (2, 4, 8)
            if not (k.startswith("chunk") and not nt)]  # the chunk kernels (x4, x8) are non-temporal only
    arms.append(("sdma", False, 8))  # the copy engine, for reference
    probe.warmup(0, 100.0)
    got = {arm: [] for arm in arms}
    for _ in range(a.rounds):
        for arm in arms:
            k, nt, b = arm
            r = probe.copy_bw(0, 0, a.bytes, a.iters, 2, kind=k, nontemporal=nt, blocks_per_cu=b)
            if not r["ok"]:
                print(json.dumps({"kind": k, "nontemporal": nt, "blocks_per_cu": b, "error": "verification failed"}))
                return 1
            got[arm].append(float(r["gbps"]))
    rows = []
    for (k, nt, b), v in got.items():
        row = {"kind": k, "nontemporal": nt, "blocks_per_cu": b, "gbps": round(statistics.median(v), 1),
               "traffic_tbps": round(2 * statistics.median(v) / 1000, 2), "runs": [round(x, 1) for x in v]}
        rows.append(row)
        print(json.dumps(row))
    best = max(rows, key=lambda r: r["gbps"])
    print(json.dumps({"best": best, "bytes": a.bytes}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
