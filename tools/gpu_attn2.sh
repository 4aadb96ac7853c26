#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step attn_bench 300 python bench/attn_bench.py --b 2 --s 4096
step attn_bench_b4 300 python bench/attn_bench.py --b 4 --s 4096
step llama8b_hip 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --attn hip --out gpurun_out/llama8b_b4_hip.json
mkdir -p gpurun_out/prof_llama_hip
step prof_llama_hip 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama_hip -o llama -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 2 --warmup 1
echo "== done"
