#!/bin/bash
# SwiGLU backward with fused transposed output: numerics + kernel timing.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_fused 600 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
step swiglu_t_bench 300 python bench/swiglu_t_bench.py
echo "== done"
