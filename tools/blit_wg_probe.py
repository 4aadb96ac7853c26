"""k=1 RCCL all-reduce (a device-to-device blit in the HIP runtime) at 2 GiB vs the K3 HBM copy
probe, under the current environment.  Run once per DEBUG_CLR_LIMIT_BLIT_WG value (read at HIP init)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gpu_topology_on_k8s_amd._native import load  # noqa: E402
from gpu_topology_on_k8s_amd.ops import probe  # noqa: E402

rccl = load("_rccl")
probe.warmup(0, 20.0)
pts = rccl.local_sweep([0], [2 << 30], "bf16", 20, 5, False, True)
cp = probe.copy_bw(0, 0, 2 << 30, iters=10, warmup_iters=2)
print(json.dumps({"limit_blit_wg": os.environ.get("DEBUG_CLR_LIMIT_BLIT_WG", "default"),
                  "rccl_k1_algbw": round(pts[0]["algbw_gbps"], 1), "wrong": pts[0]["wrong"],
                  "k3_copy_gbps": round(cp["gbps"], 1)}))
