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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--target", default="_fused")
    ap.add_argument("--out", default="/tmp/gtk_isa.s")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    from gpu_topology_on_k8s_amd._native import build

    t = next(x for x in build.targets() if x.name == a.target)
    src = Path(a.src).resolve()
    flags = [f for f in t.compile_flags() if f not in ("-fPIC",)]
    cmd = flags + t.src_flags.get(src.name, []) + ["--cuda-device-only", "-S", str(src), "-o", a.out]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        print(p.stderr[-3000:])
        return p.returncode
    text = Path(a.out).read_text()
    # per-kernel sections: from the symbol label to its .size directive
    for m in re.finditer(r"^(_Z\w+):[^\n]*$(.*?)^\s*\.size\s+\1,", text, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if a.kernel and a.kernel not in name:
            continue
        meta = {}
        for key in ("NumVgprs", "NumAgprs", "TotalNumSgprs", "ScratchSize", "LDSByteSize", "Occupancy"):
            mm = re.search(rf";\s*{key}:\s*(\d+)", text[m.end():m.end() + 4000])
            meta[key] = int(mm.group(1)) if mm else None
        ins = [ln.strip().split()[0] for ln in body.splitlines() if ln.strip() and not ln.strip().startswith((";", ".", "_"))
               and not ln.strip().endswith(":")]
        count = lambda pre: sum(1 for i in ins if i.startswith(pre))  # noqa: E731
        print(f"{name[:90]}\n  {meta}\n  mfma {count('v_mfma')}  ds_read {count('ds_read')}  accvgpr_read "
              f"{count('v_accvgpr_read')}  accvgpr_write {count('v_accvgpr_write')}  accvgpr_mov {count('v_accvgpr_mov')}  "
              f"s_waitcnt {count('s_waitcnt')}  scratch {count('scratch_')}  total {len(ins)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
