#!/bin/bash
# Llama-3-8B b4 x 4096 with every current kernel: throughput + per-kernel profile of a step.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step llama_final 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 8 --warmup 2 --placements best --out gpurun_out/llama8b_b4_final.json
step prof_llama_final 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama_final -o llama -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 2 --warmup 1
echo "== done"
