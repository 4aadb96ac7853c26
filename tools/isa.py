#!/usr/bin/env python3
"""gfx950 ISA of one source of a native target, with the build's own flags, and a register / loop
summary per kernel:

    python tools/isa.py csrc/ops/attention.hip [--target _fused] [--out /tmp/attn.s] [--kernel dkdv]

Prints, per kernel whose name matches ``--kernel``: VGPRs, AGPRs, SGPRs, scratch bytes, LDS bytes and
instruction counts (MFMA, ds_read, VALU accumulator moves, s_waitcnt) -- the numbers the kernel
docstrings quote.
"""
import argparse
import re
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


def kernel_stats(src: str, target: str = "_fused", out: str = "/tmp/gtk_isa.s") -> dict:
    """{kernel symbol: {NumVgprs, NumAgprs, TotalNumSgprs, ScratchSize, LDSByteSize, Occupancy, mfma,
    ds_read, accvgpr_read, accvgpr_write, accvgpr_mov, s_waitcnt, scratch, total}} of one source."""
    from gpu_topology_on_k8s_amd._native import build

    t = next(x for x in build.targets() if x.name == target)
    path = Path(src).resolve()
    flags = [f for f in t.compile_flags() if f not in ("-fPIC",)]
    cmd = flags + t.src_flags.get(path.name, []) + ["--cuda-device-only", "-S", str(path), "-o", out]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(p.stderr[-3000:])
    text = Path(out).read_text()
    res = {}
    for m in re.finditer(r"^(_Z\w+):[^\n]*$(.*?)^\s*\.size\s+\1,", text, re.S | re.M):
        name, body = m.group(1), m.group(2)
        meta = {}
        for key in ("NumVgprs", "NumAgprs", "TotalNumSgprs", "ScratchSize", "LDSByteSize", "Occupancy"):
            mm = re.search(rf";\s*{key}:\s*(\d+)", text[m.end():m.end() + 4000])
            meta[key] = int(mm.group(1)) if mm else None
        ins = [ln.strip().split()[0] for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", ".", "_"))
               and not ln.strip().endswith(":")]
        for k, pre in (("mfma", "v_mfma"), ("ds_read", "ds_read"), ("accvgpr_read", "v_accvgpr_read"),
                       ("accvgpr_write", "v_accvgpr_write"), ("accvgpr_mov", "v_accvgpr_mov"), ("s_waitcnt", "s_waitcnt"),
                       ("scratch", "scratch_")):
            meta[k] = sum(1 for i in ins if i.startswith(pre))
        meta["total"] = len(ins)
        res[name] = meta
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--target", default="_fused")
    ap.add_argument("--out", default="/tmp/gtk_isa.s")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    try:
        stats = kernel_stats(a.src, a.target, a.out)
    except RuntimeError as e:
        print(e)
        return 1
    for name, st in stats.items():
        if a.kernel and a.kernel not in name:
            continue
        meta = {k: st[k] for k in ("NumVgprs", "NumAgprs", "TotalNumSgprs", "ScratchSize", "LDSByteSize", "Occupancy")}
        print(f"{name[:90]}\n  {meta}\n  mfma {st['mfma']}  ds_read {st['ds_read']}  accvgpr_read {st['accvgpr_read']}  "
              f"accvgpr_write {st['accvgpr_write']}  accvgpr_mov {st['accvgpr_mov']}  s_waitcnt {st['s_waitcnt']}  "
              f"scratch {st['scratch']}  total {st['total']}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
