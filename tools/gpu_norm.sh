#!/bin/bash
# Overlapped per-bucket gradient norm: GPU tests, Llama-3-8B A/B against the serial norm.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_norm 600 python -u -m pytest tests/test_fused_gpu.py tests/test_checkpoint.py -m gpu -x -v --timeout 300 --timeout-method thread
T="python -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 8 --warmup 2"
step llama8b_norm_overlap 400 $T --overlap-norm
step llama8b_norm_serial 400 $T
echo "== done"
