#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step attn_tests 300 python -m pytest tests/test_attention_gpu.py -x -q -p no:cacheprovider
step attn_bench_b4 300 python bench/attn_bench.py --b 4 --s 4096
echo "== done"
