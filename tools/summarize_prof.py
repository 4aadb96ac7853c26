#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + PMC counter collections) into one markdown file.

    python tools/summarize_prof.py gpurun_out/prof_probe gpurun_out/pmc_lds gpurun_out/pmc_mem ... > profiles/x/SUMMARY.md

PMC rows are aggregated per kernel name (sum over dispatches); derived metrics:
  * LDS bank-conflict ratio = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  * HBM bytes = (TCC_EA0_RDREQ + TCC_EA0_WRREQ) * 64  (MI355X_MICROARCH: FETCH counts 64 B per request;
    wide streaming reads are 128-B requests tallied at 64 B, so reads are doubled for dwordx4 streams)
  * effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time
  * MFMA-busy / SQ-busy raw cycle ratio (normalisation of SQ_BUSY_CYCLES on gfx950 is uncalibrated)
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if "(" in name:
        name = name[: name.index("(")]
    return name.replace("void ", "")[:70]


def db_tables(d: str):
    """rocprofv3 >= 7 writes a rocpd SQLite database (``*.db``) by default: its ``kernels`` view has
    one row per dispatch (start/end in ns)."""
    import sqlite3

    out = []
    for f in sorted(glob.glob(os.path.join(d, "*.db"))):
        c = sqlite3.connect(f)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        if not {"name", "start", "end"} <= set(cols):
            continue
        rows = c.execute("select name, count(*), avg(end - start), min(end - start), max(end - start), sum(end - start) "
                         "from kernels group by name order by sum(end - start) desc").fetchall()
        total = sum(r[5] for r in rows) or 1
        out.append(f"### Kernel stats: `{os.path.relpath(f)}`\n")
        out.append("| kernel | calls | avg µs | min µs | max µs | % time |\n|---|---|---|---|---|---|")
        for name, n, avg, mn, mx, tot in rows:
            out.append(f"| {short(name)} | {n} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | {100 * tot / total:.1f} |")
        out.append("")
    return out


def stats_tables(d: str):
    out = db_tables(d)
    for f in sorted(glob.glob(os.path.join(d, "*kernel_stats.csv"))):
        rows = list(csv.DictReader(open(f)))
        out.append(f"### Kernel stats: `{os.path.relpath(f)}`\n")
        out.append("| kernel | calls | avg µs | min µs | max µs | % time |\n|---|---|---|---|---|---|")
        for r in rows:
            out.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['MinNs'])/1e3:.1f} | "
                       f"{float(r['MaxNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
        out.append("")
    return out


def _db_counter_rows(f: str):
    """rocpd database: the ``counters_collection`` view, one row per (dispatch, counter), mapped onto
    the CSV column names the aggregation below reads."""
    import sqlite3

    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    if "counter_name" not in cols:
        return []
    q = ("select kernel_name, counter_name, value, dispatch_id, start, end, grid_size, workgroup_size, lds_block_size, "
         "vgpr_count, accum_vgpr_count, sgpr_count from counters_collection")
    keys = ("Kernel_Name", "Counter_Name", "Counter_Value", "Dispatch_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size",
            "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")
    return [dict(zip(keys, r)) for r in c.execute(q)]


def pmc_tables(d: str):
    out = []
    sources = [(f, list(csv.DictReader(open(f)))) for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv")))]
    sources += [(f, rows) for f in sorted(glob.glob(os.path.join(d, "*.db"))) for rows in [_db_counter_rows(f)] if rows]
    for f, rows in sources:
        agg = defaultdict(lambda: defaultdict(float))
        meta = {}
        wall = defaultdict(float)
        seen = set()
        for r in rows:
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            did = (r["Dispatch_Id"], k)
            if did not in seen:
                seen.add(did)
                wall[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                agg[k]["_dispatches"] += 1
            meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"])
        counters = sorted({c for v in agg.values() for c in v if not c.startswith("_")})
        out.append(f"### PMC: `{os.path.relpath(f)}`\n")
        out.append("| kernel | dispatches | grid | wg | LDS B | VGPR | AGPR | SGPR | " + " | ".join(counters) + " | derived |")
        out.append("|" + "---|" * (9 + len(counters)))
        for k, v in agg.items():
            der = []
            if v.get("SQ_LDS_IDX_ACTIVE"):
                der.append(f"LDS conflict {v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_LDS_IDX_ACTIVE'] * 100:.2f}%")
            if "TCC_EA0_RDREQ_sum" in v and wall[k] > 0:
                rd = v["TCC_EA0_RDREQ_sum"] * 64 * 2  # 128-B requests counted at 64 B for wide streams
                wr = v.get("TCC_EA0_WRREQ_sum", 0) * 64
                der.append(f"HBM ≈{(rd + wr) / wall[k] / 1e9:.0f} GB/s (rd {rd/1e9:.2f} GB, wr {wr/1e9:.2f} GB)")
            if v.get("GRBM_GUI_ACTIVE") and wall[k] > 0:
                der.append(f"clk ≈{v['GRBM_GUI_ACTIVE'] / 8 / wall[k] / 1e9:.2f} GHz")
            if v.get("SQ_VALU_MFMA_BUSY_CYCLES") and v.get("SQ_BUSY_CYCLES"):
                der.append(f"MFMA-busy/SQ-busy cycles {v['SQ_VALU_MFMA_BUSY_CYCLES'] / v['SQ_BUSY_CYCLES']:.2f} (raw ratio)")
            m = meta[k]
            out.append(f"| {k} | {int(v['_dispatches'])} | {m[0]} | {m[1]} | {m[2]} | {m[3]} | {m[4]} | {m[5]} | "
                       + " | ".join(f"{v.get(c, 0):.3g}" for c in counters) + f" | {'; '.join(der)} |")
        out.append("")
    return out


def main(dirs):
    lines = ["# rocprofv3 summary", ""]
    for d in dirs:
        lines += stats_tables(d) + pmc_tables(d)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1:])
