#!/bin/bash
# Full GPU tier + smoke + headline bench + training profile.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 300 python bench.py
mkdir -p gpurun_out/prof_llama_v2
step prof_llama_v2 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_llama_v2 -o llama -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 2 --warmup 1
echo "== done"
