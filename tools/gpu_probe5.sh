#!/bin/bash
# K5 gather kernel + probe CLI ingress stage + bench on one GPU.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_native 600 python -u -m pytest tests/test_gpu_native.py -m gpu -x -v --timeout 300 --timeout-method thread
step bench_k1 300 python3 bench.py --steps 50 --warmup 10
echo "== done"
