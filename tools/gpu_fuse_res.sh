#!/bin/bash
# Fused residual add + RMSNorm: numerics tests, then Llama-3-8B A/B (fused default vs --no-fuse-residual).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_fused 600 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
T="python -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 6 --warmup 2"
step llama8b_fused 400 $T
step llama8b_unfused 400 $T --no-fuse-residual
echo "== done"
