#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step attn_tests 300 python -m pytest tests/test_attention_gpu.py -x -q -p no:cacheprovider
step attn_bench_b4 300 python bench/attn_bench.py --b 4 --s 4096
step llama8b_hip 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --attn hip --out gpurun_out/llama8b_b4_hip.json
echo "== done"
