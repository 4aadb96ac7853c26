#!/bin/bash
# GPU tests + smoke + Llama-3-8B single-GPU training throughput + rocprofv3 kernel stats of a step.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step llama8b_b2 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 2 --seq 4096 --steps 4 --warmup 2 --placements best --out gpurun_out/llama8b_b2.json
step llama8b_b4 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --out gpurun_out/llama8b_b4.json
step prof_llama 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama -o llama -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 2 --seq 4096 --steps 2 --warmup 1
echo "== done"
