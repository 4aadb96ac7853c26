#!/bin/bash
# attention kernels: GPU tests + timing + kernel stats (quick A/B loop).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_attn 400 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step attn_bench 200 python bench/attn_bench.py --b 4 --s 4096 --iters 10
step attn_prof 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn_q -o attn -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 5
echo "== done"
