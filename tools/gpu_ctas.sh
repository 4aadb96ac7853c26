#!/bin/bash
# RCCL communicator config path (ncclConfig_t minCTAs/maxCTAs) + bench tuning pass at k=1.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step bench_k1_tune 300 env NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT python3 bench.py --steps 50 --warmup 10 --ctas tune
grep -i "min ctas\|max ctas\|Channel 00" gpurun_out/bench_k1_tune.log | head -20
echo "== done"
