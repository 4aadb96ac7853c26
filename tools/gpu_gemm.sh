#!/bin/bash
# hipBLASLt GEMM throughput at the Llama-3-8B training shapes.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step gemm_bench 300 python bench/gemm_bench.py --tokens 16384 --iters 10
echo "== done"
