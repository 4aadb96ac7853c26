#!/bin/bash
# forward running-max slack: attention GPU tests, kernel timing, then the Llama-3-8B step.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_attn 300 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step attn_bench 200 python bench/attn_bench.py --b 4 --s 4096 --iters 10
step llama_slack 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 8 --warmup 2 --placements best --out gpurun_out/llama8b_b4_slack.json
echo "== done"
