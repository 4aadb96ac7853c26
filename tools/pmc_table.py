#!/usr/bin/env python3
"""Per-kernel counter table from a rocprofv3 ``--pmc`` run database (rocpd SQLite).

    python tools/pmc_table.py gpurun_out/x/pmc/run_results.db [--filter attn]

Sums every counter over a kernel's dispatches and prints a markdown table with the derived ratios
used in profiles/: MFMA busy per GUI cycle (``SQ_VALU_MFMA_BUSY_CYCLES`` is summed over the chip's
1024 SIMDs and ``GRBM_GUI_ACTIVE`` over its 8 XCDs, so a full MFMA pipe reads 128) and LDS waits per
wave cycle (``SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES``).
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select k.name, p.counter_name, sum(p.counter_value), count(distinct k.dispatch_id), avg(k.duration) "
                     "from pmc_events p join kernels k on p.dispatch_id = k.dispatch_id group by k.name, p.counter_name")
    agg = defaultdict(dict)
    meta = {}
    for name, ctr, val, n, dur in rows:
        short = name.split("(")[0].replace("void ", "")[:60]
        if a.filter and a.filter not in short:
            continue
        agg[short][ctr] = agg[short].get(ctr, 0.0) + float(val)
        meta[short] = (n, dur)
    ctrs = sorted({k for d in agg.values() for k in d})
    mem = any("TCC_EA0_RDREQ_sum" in d for d in agg.values())
    extra = " | EA GB per dispatch (lower bound) | EA TB/s (lower bound)" if mem else ""
    print("| kernel | dispatches | avg µs | " + " | ".join(ctrs) + " | MFMA busy / GUI cycle (of 128) | LDS waits / wave cycles"
          + extra + " |")
    print("|---|---|---|" + "---|" * len(ctrs) + "---|---|" + ("---|---|" if mem else ""))
    for k, d in sorted(agg.items(), key=lambda x: -meta[x[0]][1] * meta[x[0]][0]):
        n, dur = meta[k]
        busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / d["GRBM_GUI_ACTIVE"] if d.get("GRBM_GUI_ACTIVE") else None
        ldsw = d.get("SQ_WAIT_INST_LDS", 0) / d["SQ_WAVE_CYCLES"] if d.get("SQ_WAVE_CYCLES") else None
        cells = " | ".join(f"{d.get(x, 0):.3g}" for x in ctrs)
        tail = ""
        if mem:  # memory-side requests x 64 B: a 128-B streaming read is tallied once, so reads count half
            gb = (d.get("TCC_EA0_RDREQ_sum", 0) + d.get("TCC_EA0_WRREQ_sum", 0)) * 64 / n / 1e9
            tail = f" | {gb:.3f} | {gb / (dur / 1e9) / 1e3:.2f}" if dur else " | | "
        print(f"| {k} | {n} | {dur / 1e3:.1f} | {cells} | "
              f"{'' if busy is None else f'{busy:.1f} ({busy / 128:.0%})'} | {'' if ldsw is None else f'{ldsw:.1%}'}{tail} |")


if __name__ == "__main__":
    main()
