#!/bin/bash
# dK/dV v4 (software-pipelined slices): bitwise vs v3, timing, PMC.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_attn 400 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread
step attn_bench_v4 200 python bench/attn_bench.py --b 4 --s 4096 --iters 10
step attn_prof_v4 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn_v4 -o attn -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 5
step attn_pmc_v4 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn_v4 -o pmc -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 2
echo "== done"
