#!/bin/bash
# RMSNorm backward at 2 waves/SIMD: numerics, kernel timing, Llama-3-8B step.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_norm_grid 300 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v -k "rmsnorm or fused_residual or llama" --timeout 120 --timeout-method thread
step norm_bench_grid 120 python3 bench/norm_bench.py
step llama8b_grid 400 python -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 8 --warmup 2
echo "== done"
