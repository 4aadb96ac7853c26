#!/usr/bin/env python3
"""Workload for one rocprofv3 --pmc pass over the HIP attention kernels, with the K4 / K4r MFMA loops
as the calibration of "MFMA busy" (K4 keeps the MFMA pipe full by construction):

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE ... -- python3 tools/pmc_attn.py

Llama-3-8B shape: B 4, 32 q-heads / 8 kv-heads, S 4096, D 128, causal; 3 forward + 3 backward calls.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402
from gpu_topology_on_k8s_amd.ops.probe import warmup  # noqa: E402


def main():
    warmup(0, 100.0)
    warmup(0, 100.0, random_operands=True)
    B, H, Hkv, S, D = 4, 32, 8, 4096, 128
    torch.manual_seed(0)
    q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, S, D, device="cuda", dtype=torch.bfloat16)
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    hip = fused.hip()
    variants = [getattr(hip, n) for n in sorted(dir(hip)) if n.startswith("attn_bwd_")]  # A/B builds only
    for _ in range(3):
        o, lse = hip.attn_fwd(q, k, v, D ** -0.5)
        hip.attn_bwd(do, q, k, v, o, lse, D ** -0.5)
        for fn in variants:
            fn(do, q, k, v, o, lse, D ** -0.5)
        for n in sorted(dir(hip)):
            if n.startswith("attn_fwdv_"):
                getattr(hip, n)(q, k, v, D ** -0.5)
    torch.cuda.synchronize()
    print("pmc_attn done", flush=True)


if __name__ == "__main__":
    main()
