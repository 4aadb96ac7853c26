#!/bin/bash
# Extend the TunableOp table with the NT-layout backward GEMM shapes (merged into a copy of the shipped table).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cp gpu_topology_on_k8s_amd/models/tuned/tunableop_mi355x.csv gpurun_out/tunableop_mi355x_nt.csv
( while sleep 50; do date >> gpurun_out/tune_heartbeat.log; done ) &
HB=$!
step gemm_tune_nt 1050 python -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 1 --warmup 1 --gemm-tuning tune --gemm-table gpurun_out/tunableop_mi355x_nt.csv --gemm-layout nt
kill $HB
wc -l gpurun_out/tunableop_mi355x_nt.csv
echo "== done"
