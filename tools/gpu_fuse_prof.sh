#!/bin/bash
# Kernel stats of Llama-3-8B steps with the fused residual add+RMSNorm vs separate adds.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
A="--model llama3-8b --batch 4 --seq 4096 --steps 2 --warmup 1"
step prof_fused 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fused -o run -- python3 -m gpu_topology_on_k8s_amd.models.train $A
step prof_unfused 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_unfused -o run -- python3 -m gpu_topology_on_k8s_amd.models.train $A --no-fuse-residual
echo "== done"
