#!/bin/bash
# attention forward v3 A/B: numerics tests, then timing + kernel stats vs forward v2.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_fwd3 300 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q -k "fwd_v3 or forward" --timeout 120 --timeout-method thread
step attn_bench 200 python bench/attn_bench.py --b 4 --s 4096 --iters 10
step attn_bench_s8k 200 python bench/attn_bench.py --b 1 --s 8192 --iters 10
step attn_prof 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fwd3 -o attn -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 5
echo "== done"
