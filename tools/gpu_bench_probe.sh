#!/bin/bash
# bench.py end to end on one GPU: child-process link probe -> placement -> RCCL all-reduce.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_bench 400 python -u -m pytest tests/test_gpu_native.py -m gpu -x -v --timeout 200 --timeout-method thread -k "bench"
step bench_k1_probe 300 python3 bench.py --steps 50 --warmup 10
echo "== done"
