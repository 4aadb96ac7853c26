#!/bin/bash
# rocprofv3 evidence for the probe kernels and the bench (CSV summaries under gpurun_out/prof_*).
#   gpurun --timeout 1100 -- bash tools/gpu_profile.sh
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step counters_list 120 rocprofv3 -L
step prof_bench 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 20 --warmup 5
step prof_probe 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_probe -o probe -- python3 bench/probe_bench.py --sizes 256,1024 --iters 5 --out gpurun_out/probe_sweep.json
step pmc_probe_lds 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_lds -o pmc -- python3 bench/probe_bench.py --sizes 256 --iters 3
step pmc_probe_mem 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmc_mem -o pmc -- python3 bench/probe_bench.py --sizes 256 --iters 3
step pmc_probe_mfma 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma -o pmc -- python3 bench/probe_bench.py --sizes 64 --iters 3
echo "== done"
