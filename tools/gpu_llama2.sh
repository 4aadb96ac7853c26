#!/bin/bash
# Llama-3-8B single-GPU training throughput (b4 x 4096) + rocprofv3 kernel stats of a step + attention kernel split.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step llama8b_b4 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --out gpurun_out/llama8b_b4.json
step prof_llama 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama3 -o llama -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 2 --warmup 1
step attn_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn3 -o attn -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 5
step gemm_bench 300 python bench/gemm_bench.py --tokens 16384 --iters 10
echo "== done"
