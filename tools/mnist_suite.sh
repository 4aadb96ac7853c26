#!/usr/bin/env bash
# MNIST CNN (Gaia Exp. 6 workload) on one MI355X: eager vs hipGraph step over batch sizes, then a
# rocprofv3 kernel trace of the graph step.  Usage: bash tools/mnist_suite.sh <outdir>
set -euo pipefail
out=${1:-gpurun_out/mnist}
mkdir -p "$out"
export TMPDIR=/tmp
for b in 64 256 1024; do
  for conv in torch hip; do
    for g in off on; do
      timeout -k 10 300 python -m gpu_topology_on_k8s_amd.models.train --model mnist-cnn --batch "$b" --steps 200 --warmup 5 \
        --graph "$g" --conv "$conv" --gemm-tuning off > "$out/train_b${b}_${conv}_graph_${g}.json" 2> "$out/train_b${b}_${conv}_graph_${g}.err"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o mnist -- python3 -m gpu_topology_on_k8s_amd.models.train \
  --model mnist-cnn --batch 64 --steps 200 --warmup 5 --graph on --gemm-tuning off > "$out/prof.log" 2>&1
