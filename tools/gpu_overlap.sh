#!/bin/bash
# NT operand transposes on a side stream in forward: numerics + Llama-3-8B A/B (overlap vs in-backward).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_fused 600 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
step llama_overlap 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 6 --warmup 2 --placements best --overlap-transposes --out gpurun_out/llama8b_b4_overlap.json
step llama_no_overlap 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 6 --warmup 2 --placements best --out gpurun_out/llama8b_b4_no_overlap.json
echo "== done"
