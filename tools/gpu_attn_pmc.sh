#!/bin/bash
# PMC counters of the attention kernels (what bounds dK/dV v3, dQ v2, fwd v2).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step attn_pmc1 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn1 -o pmc -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 2
step attn_pmc2 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_attn2 -o pmc -- python3 bench/attn_bench.py --b 4 --s 4096 --iters 2
echo "== done"
