#!/bin/bash
# One gpurun call: GPU tests, default bench, rocprofv3 kernel stats of the bench.
#   gpurun --timeout 1100 -- bash tools/gpu_validate.sh
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step bench_default 300 python bench.py
step bench_torch 300 python bench.py --backend torch --steps 20 --warmup 5
mkdir -p gpurun_out/prof_bench
step rocprof_bench 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 20 --warmup 5
echo "== done"
