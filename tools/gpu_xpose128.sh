#!/bin/bash
# 128-row transpose / swiglu_bwd_t tiles: exactness tests, timing, LDS-conflict + HBM counters.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_xpose 300 python -u -m pytest tests/test_fused_gpu.py -m gpu -x -q -k "transpose or swiglu" --timeout 120 --timeout-method thread
step swiglu_t_bench 200 python bench/swiglu_t_bench.py
step pmc_xpose_lds 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_xpose128_lds -o pmc -- python3 bench/swiglu_t_bench.py
step pmc_xpose_mem 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_xpose128_mem -o pmc -- python3 bench/swiglu_t_bench.py
echo "== done"
