#!/bin/bash
# Fused residual add + RMSNorm (dres prefetched): numerics, kernel stats, Llama-3-8B A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_fused 600 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
A="--model llama3-8b --batch 4 --seq 4096 --steps 2 --warmup 1"
step prof_fused2 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused2 -o run -- python3 -m gpu_topology_on_k8s_amd.models.train $A
T="python -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 8 --warmup 2"
step llama8b_fused2 400 $T
step llama8b_unfused2 400 $T --no-fuse-residual
echo "== done"
