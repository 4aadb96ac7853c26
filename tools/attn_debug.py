#!/usr/bin/env python3
"""Diagnose the HIP attention forward's QK^T stage: compare the raw S^T accumulator dump of the
first KV tile with exact integer dot products and identify which (query, key) each value really is."""
import sys

import torch

sys.path.insert(0, ".")
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def crow(i, hh):
    return (i & 3) + 8 * (i >> 2) + 4 * hh


def tr_probe():
    rows = torch.arange(64, device="cuda").view(64, 1).expand(64, 128).to(torch.bfloat16).contiguous()
    cols = torch.arange(128, device="cuda").view(1, 128).expand(64, 128).to(torch.bfloat16).contiguous()
    bad = 0
    for t in range(4):
        for col0 in (0, 32, 64, 96):
            gr = fused.hip().attn_tr_probe(rows, t, col0).float().cpu()
            gc = fused.hip().attn_tr_probe(cols, t, col0).float().cpu()
            for lane in range(64):
                r, hh = lane & 31, lane >> 5
                for j in range(8):
                    want_row = 16 * t + 8 * (j >> 2) + 4 * hh + (j & 3)
                    want_col = col0 + r
                    if (gr[lane, j], gc[lane, j]) != (want_row, want_col):
                        if bad < 12:
                            print(f"tr t={t} col0={col0} lane={lane} j={j}: got (row {gr[lane, j]:.0f}, col {gc[lane, j]:.0f})"
                                  f" want ({want_row}, {want_col})")
                        bad += 1
    print("tr_frag mismatches:", bad)
    gr = fused.hip().attn_tr_probe(rows, 0, 0).float().cpu()
    gc = fused.hip().attn_tr_probe(cols, 0, 0).float().cpu()
    for lane in list(range(0, 20)) + [32, 33, 36, 48]:
        print(f"lane {lane:2d}: " + " ".join(f"({gr[lane, j]:.0f},{gc[lane, j]:.0f})" for j in range(8)))


def main():
    tr_probe()
    torch.manual_seed(0)
    B, H, Hkv, S = 1, 1, 1, 128
    q = torch.randint(-3, 4, (B, H, S, 128), device="cuda").to(torch.bfloat16)
    k = torch.randint(-3, 4, (B, Hkv, S, 128), device="cuda").to(torch.bfloat16)
    v = torch.randn(B, Hkv, S, 128, device="cuda").to(torch.bfloat16)
    o, lse, dbg = fused.hip().attn_fwd_debug(q, k, v, 128 ** -0.5)
    full = (q[0, 0].float() @ k[0, 0].float().T).cpu()  # [query, key]
    dbg = dbg.cpu()
    ok = bad = 0
    examples = []
    lookup = {}
    for qi in range(S):
        for ki in range(64):
            lookup.setdefault(float(full[qi, ki]), []).append((qi, ki))
    for w in range(4):
        for lane in range(64):
            r, hh = lane & 31, lane >> 5
            for i in range(32):
                sub, reg = i // 16, i % 16
                qq, kk = w * 32 + r, sub * 32 + crow(reg, hh)
                got = float(dbg[0, 0, w, lane, i])
                if got == float(full[qq, kk]):
                    ok += 1
                else:
                    bad += 1
                    if len(examples) < 12:
                        examples.append((w, lane, i, qq, kk, got, float(full[qq, kk]), lookup.get(got, [])[:4]))
    print(f"S^T dump: {ok} match, {bad} mismatch")
    for e in examples:
        print("w=%d lane=%d reg=%d expect(q=%d,k=%d) got=%g want=%g  got-matches(q,k)=%s" % e)
    ref = fused.attention_ref(q, k, v)
    print("o rel err", ((o.float() - ref.float()).norm() / ref.float().norm()).item())
    rows = ((o.float() - ref.float()).abs().amax(dim=(2, 3))[0] > 0.05).nonzero().flatten().tolist()
    print("bad output rows:", rows[:40], "count", len(rows))


if __name__ == "__main__":
    main()
