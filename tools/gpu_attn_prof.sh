#!/bin/bash
# Per-kernel time and counters for the HIP attention kernels at the Llama-3-8B shape.
#   gpurun --timeout 900 -- bash tools/gpu_attn_prof.sh
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step attn_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn -o attn -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 5
step attn_pmc_lds 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn_lds -o pmc -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 2
step attn_pmc_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn_mfma -o pmc -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 2
echo "== done"
