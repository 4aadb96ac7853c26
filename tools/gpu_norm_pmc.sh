#!/bin/bash
# Fused add+RMSNorm kernels at the Llama-3-8B shape: timing (HBM-streaming buffers) and HBM traffic counters.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step norm_bench 120 python3 bench/norm_bench.py
step pmc_norm_mem 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_norm_mem -o pmc -- python3 bench/norm_bench.py
echo "== done"
