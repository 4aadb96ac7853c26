#!/bin/bash
# hipGraph-captured RCCL all-reduce: GPU tests of the capture path, then the k=1 bench (its JSON
# carries the eager vs graph small-message latency table).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_rccl 600 python -u -m pytest tests/test_gpu_native.py -m gpu -x -v -k "rccl or bench_py" --timeout 300 --timeout-method thread
step bench_k1_graph 300 python3 bench.py --steps 50 --warmup 10
echo "== done"
