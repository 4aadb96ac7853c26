#!/bin/bash
# ZeRO-1 path on the GPU: sharded-AdamW kernel test, then Llama-3-8B b4 with and without --zero1.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_zero1 300 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "adamw"
step llama_zero1 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 6 --warmup 2 --placements best --zero1 --out gpurun_out/llama8b_b4_zero1.json
step llama_base 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 6 --warmup 2 --placements best --out gpurun_out/llama8b_b4_base.json
echo "== done"
