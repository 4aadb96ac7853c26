#!/bin/bash
# hipBLASLt backward-GEMM layouts at the Llama-3-8B shapes: as autograd issues them vs NT + transposes.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step gemm_layout 300 python -u bench/gemm_layout_bench.py --tokens 16384 --iters 10
step gemm_layout_tuned 700 python -u bench/gemm_layout_bench.py --tokens 16384 --iters 10 --tune
echo "== done"
