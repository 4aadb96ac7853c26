#!/bin/bash
# GPU tests + Llama-3-8B b4 bench after the direct weight-gradient change; then extend the TunableOp table.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step llama8b_b4 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --out gpurun_out/llama8b_b4_direct.json
cp gpu_topology_on_k8s_amd/models/tuned/tunableop_mi355x.csv gpurun_out/tunableop_mi355x.csv
( while sleep 60; do date >> gpurun_out/tune_heartbeat.log; done ) &
HB=$!
step gemm_tune 900 python -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 1 --warmup 1 --gemm-tuning tune --gemm-table gpurun_out/tunableop_mi355x.csv
kill $HB
step llama8b_b4_tuned 600 python bench/train_llama.py --gpus 1 --model llama3-8b --batch 4 --seq 4096 --steps 4 --warmup 2 --placements best --gemm-tuning use --gemm-table gpurun_out/tunableop_mi355x.csv --out gpurun_out/llama8b_b4_direct_tuned.json
echo "== done"
