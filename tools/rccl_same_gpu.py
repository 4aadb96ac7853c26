#!/usr/bin/env python3
"""Can RCCL run a communicator whose ranks share one GPU?  (the one-GPU box's only way to execute
the k >= 2 native path).  Launch with torchrun, 2 ranks:

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
        tools/rccl_same_gpu.py

Every rank binds to HIP device 0, then tries (1) the framework's native communicator
(``_rccl.Comm``, ncclCommInitRank) with an exact-checked all-reduce, and (2) torch.distributed's
nccl backend.  Rank 0 prints one JSON line per attempt: ok, or the error RCCL gave.
"""
import json
import os
import sys
import time
from datetime import timedelta

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from gpu_topology_on_k8s_amd.parallel.allreduce import AllReduceRunner, DistEnv  # noqa: E402


def main() -> int:
    env = DistEnv.from_env()
    torch.cuda.set_device(0)
    env.store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]) + 1, env.world, env.rank == 0,
                              timedelta(seconds=60))
    out = {"rank": env.rank, "world": env.world}
    try:
        t = time.perf_counter()
        r = AllReduceRunner(env, 0, 1 << 20, "bf16", "native", tag="same-gpu")
        wrong = r.check()
        r.step()
        r.synchronize()
        r.close()
        out["native"] = {"ok": wrong == 0, "wrong": wrong, "s": round(time.perf_counter() - t, 2)}
    except Exception as e:  # noqa: BLE001 - the answer is the error
        out["native"] = {"ok": False, "error": str(e)[-300:]}
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0), timeout=timedelta(seconds=60))
        x = torch.full((1 << 18,), float(env.rank + 1), device="cuda:0")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        want = env.world * (env.world + 1) / 2
        out["torch_nccl"] = {"ok": bool((x == want).all().item())}
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        out["torch_nccl"] = {"ok": False, "error": str(e)[-300:]}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
