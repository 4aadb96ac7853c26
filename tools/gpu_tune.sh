#!/bin/bash
# TunableOp: time every hipBLASLt/rocBLAS solution for the Llama-3-8B b4 x 4096 step's GEMMs (resuming
# from the shipped table), then re-run the training bench reading the winners.  Copy the resulting
# gpurun_out/tunableop_mi355x.csv to gpu_topology_on_k8s_amd/models/tuned/.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cp gpu_topology_on_k8s_amd/models/tuned/tunableop_mi355x.csv gpurun_out/tunableop_mi355x.csv
( while sleep 60; do date >> gpurun_out/tune_heartbeat.log; wc -l gpurun_out/tunableop_mi355x.csv >> gpurun_out/tune_heartbeat.log; done ) &
HB=$!
step gemm_tune 1000 python -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 1 --warmup 1 --gemm-tuning tune --gemm-table gpurun_out/tunableop_mi355x.csv
kill $HB
step llama8b_b4_tuned 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --gemm-tuning use --gemm-table gpurun_out/tunableop_mi355x.csv --out gpurun_out/llama8b_b4_tuned.json
echo "== done"
