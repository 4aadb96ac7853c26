#!/bin/bash
# HIP transpose kernel + NT backward-GEMM layout: numerics, GEMM/transposes timing, Llama-3-8B A/B.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_fused 600 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
step gemm_layout2 300 python -u bench/gemm_layout_bench.py --tokens 16384 --iters 10
step llama_nt 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --gemm-layout nt --out gpurun_out/llama8b_b4_nt.json
step llama_native 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --gemm-layout native --out gpurun_out/llama8b_b4_native.json
echo "== done"
