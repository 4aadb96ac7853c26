#!/bin/bash
# smoke() + rocprofv3 counters of the HIP transpose / swiglu_bwd_t kernels (LDS bank conflicts, HBM traffic).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof_xpose 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_xpose -o xpose -- python3 bench/swiglu_t_bench.py
step pmc_xpose_lds 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_xpose_lds -o pmc -- python3 bench/swiglu_t_bench.py
step pmc_xpose_mem 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_xpose_mem -o pmc -- python3 bench/swiglu_t_bench.py
echo "== done"
