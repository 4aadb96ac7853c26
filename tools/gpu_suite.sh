#!/usr/bin/env bash
# One gpurun call per invocation:  gpurun --timeout 1200 -- 'bash tools/gpu_suite.sh <mode> <outdir>'
#   suite    pytest -m gpu, smoke(), headline bench (k=1)
#   bench    headline bench only (the driver's command line)
#   profile  rocprofv3 --kernel-trace --stats of the headline bench and of the link probe
# Every GPU step has its own time limit; the first failing step ends the call (exit status kept).
set -uo pipefail
mode=${1:-suite}
out=${2:-gpurun_out/run}
mkdir -p "$out"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0

step() {  # step <name> <seconds> <command...>
  local name=$1 secs=$2; shift 2
  echo "[gpu_suite] $name"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  tail -3 "$out/$name.log"
  if [ $rc -ne 0 ]; then echo "[gpu_suite] $name failed rc=$rc"; exit $rc; fi
}

case "$mode" in
  suite)
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread
    step smoke 300 python -u -c 'import __graft_entry__ as g; g.smoke()'
    step bench_k1 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
    ;;
  bench)
    step bench_k1 600 python -u bench.py --gpus 1 --steps 20 --warmup 5
    ;;
  profile)
    step prof_bench 600 rocprofv3 --kernel-trace --stats -d "$out/prof_bench" -o run -- python3 bench.py --steps 5 --warmup 2 --sweep off
    step prof_probe 600 rocprofv3 --kernel-trace --stats -d "$out/prof_probe" -o run -- python3 -m gpu_topology_on_k8s_amd probe --preset full
    ;;
  ring)
    # K6 concurrent ring probe: kernel stats, then LDS and memory counters, each pass in its own run
    step prof_ring 300 rocprofv3 --kernel-trace --stats -d "$out/prof_ring" -o run -- python3 -m gpu_topology_on_k8s_amd ring --devices 0,0,0 --preset full
    step pmc_ring_lds 120 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --kernel-trace -d "$out/pmc_ring_lds" -o run -- python3 -m gpu_topology_on_k8s_amd ring --devices 0,0,0 --preset full --patterns all
    step pmc_ring_mem 120 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace -d "$out/pmc_ring_mem" -o run -- python3 -m gpu_topology_on_k8s_amd ring --devices 0,0,0 --preset full --patterns all
    ;;
  ipc)
    # K1 read, K2 write and K5 gather on imported HIP IPC mappings (one JSON line each)
    for m in read write gather; do
      step "ipc_$m" 120 python -u -m gpu_topology_on_k8s_amd ipc --mode "$m" --bytes $((256 << 20))
    done
    ;;
  llama)
    # the config-5 workload on the current tree: Llama-3-8B b4 x 4096 step, then its kernel trace
    step llama8b_b4 600 python -u -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 5 --warmup 2
    step prof_llama 600 rocprofv3 --kernel-trace --stats -d "$out/prof_llama" -o run -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 3 --warmup 1
    ;;
  learn)
    # end-to-end learning at the config-5 shape: one repeated batch must be memorised, fresh uniform
    # tokens cannot be learnt below ln(vocab) (profiles/r03_learn)
    step learn_repeat 600 python -u -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 40 --warmup 0 --repeat-batch
    step learn_random 600 python -u -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 40 --warmup 0
    ;;
  cumask)
    # MFMA rate and HBM copy under HSA_CU_MASK (the time-sliced shares' spatial split, profiles/r02_cumask)
    for m in "" "0:0-127" "0:0-63" "0:0-31,128-159"; do
      echo "mask=[$m]" >> "$out/cumask.log"
      HSA_CU_MASK="$m" timeout -k 10 60 python -c 'import json
from gpu_topology_on_k8s_amd.ops import probe
w = probe.warmup(0, 200.0)
c = probe.copy_bw(0, 0, 512 << 20, 5, 1)
print(json.dumps({"tflops": round(float(w["tflops"]), 1), "hbm_copy_gbps": round(float(c["gbps"]), 1)}))' >> "$out/cumask.log" 2>&1 || exit 1
    done
    ;;
  attn)
    # attention kernels: bit-identity / determinism tests, interleaved A/B timings, MFMA-busy counters
    step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 300 --timeout-method thread
    step ab_b4 300 python -u bench/attn_bench.py --b 4 --s 4096 --iters 5 --ab 30
    step ab_b2 300 python -u bench/attn_bench.py --b 2 --s 4096 --iters 5 --ab 30
    step pmc_attn 120 timeout -s KILL 100 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS --kernel-trace -d "$out/pmc_attn" -o run -- python3 tools/pmc_attn.py
    ;;
  normpf)
    # RMSNorm backward with the next row prefetched: tests, norm bench, step, trace
    step pytest_fused 600 python -u -m pytest tests/test_fused_gpu.py -x -v --timeout 300 --timeout-method thread
    step norm_bench 300 python -u bench/norm_bench.py
    step llama 600 python -u -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 5 --warmup 2
    step prof_llama 600 rocprofv3 --kernel-trace --stats -d "$out/prof_llama" -o run -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 3 --warmup 1
    ;;
  memk)
    # memory-bound tile kernels with every load of the tile issued first: tests, kernel A/B bench, step, trace
    step pytest_fused 600 python -u -m pytest tests/test_fused_gpu.py -x -v --timeout 300 --timeout-method thread
    step fused_t_ab 300 python -u bench/fused_t_ab.py
    step adamw_t_ab 300 python -u bench/adamw_t_ab.py
    step llama 600 python -u -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 5 --warmup 2
    step prof_llama 600 rocprofv3 --kernel-trace --stats -d "$out/prof_llama" -o run -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 3 --warmup 1
    ;;
  pmcstep)
    # counters over one Llama-3-8B step: MFMA busy, then memory-side requests (each pass its own run),
    # summarised on the box (the per-dispatch databases exceed what gpurun copies back)
    step pmc_mfma 300 timeout -s KILL 290 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d "$out/mfma" -o run -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 1 --warmup 1
    step pmc_mem 300 timeout -s KILL 290 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE --kernel-trace -d "$out/mem" -o run -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 1 --warmup 1
    step pmc_tables 120 bash -c "python tools/pmc_table.py $out/mfma/run_results.db > $out/mfma.md && python tools/pmc_table.py $out/mem/run_results.db > $out/mem.md && rm -rf $out/mfma $out/mem"
    ;;
  attn_ab)
    # attention backward A/B (interleaved, B 4 and 2) with bit-identity tests and counters
    step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 300 --timeout-method thread
    step ab_b4 300 python -u bench/attn_bench.py --b 4 --ab 30
    step ab_b2 300 python -u bench/attn_bench.py --b 2 --ab 30
    step pmc_attn 120 timeout -s KILL 100 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-trace -d "$out/pmc_attn" -o run -- python3 tools/pmc_attn.py
    ;;
  attn_step)
    # round 5: attention kernel tests, the fused-op tests, then the Llama-3-8B step with this tree's
    # attention backward against the round-4 build's (scratch/r04, interleaved), and the step's trace
    step pytest_attn 600 python -u -m pytest tests/test_attention_gpu.py tests/test_fused_gpu.py -x -v --timeout 300 --timeout-method thread
    step step_ab 900 python -u bench/attn_step_ab.py --so ${AB_SO:-scratch/r04/_fused.cpython-310-x86_64-linux-gnu.so} --rounds 4 --steps 3
    step prof_llama 600 rocprofv3 --kernel-trace --stats -d "$out/prof_llama" -o run -- python3 -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 3 --warmup 1
    ;;
  r05)
    # round 5 checks: the share guard by PCI address (+ managed memory), the k >= 2 DP reduction checks
    # rehearsed on the one GPU, and the loss lineage with this tree's and the round-4 attention backward
    step pytest_r05 900 python -u -m pytest tests/test_gpu_shares.py tests/test_gpu_rehearsal.py tests/test_gpu_multi.py -k "guard or doctor or rehearsal or dp" -x -v -rP --timeout 300 --timeout-method thread
    step lineage_v7 400 python -u -m gpu_topology_on_k8s_amd.models.train --model llama3-8b --batch 4 --seq 4096 --steps 5 --warmup 2
    so=${AB_SO:-scratch/r04/_fused.cpython-310-x86_64-linux-gnu.so}  # another tree's build (git-ignored)
    if [ -f "$so" ]; then
      step lineage_r04attn 400 python -u bench/with_attn_bwd.py --so "$so" -- --model llama3-8b --batch 4 --seq 4096 --steps 5 --warmup 2
    else
      echo "[gpu_suite] lineage_r04attn skipped: no $so"
    fi
    ;;
  shadow)
    # what 8-GPU DP communication costs the Llama-3-8B step: comm-shadow CTA sweep
    step shadow_sweep 1100 python -u bench/comm_shadow_sweep.py --ctas ${SHADOW_CTAS:-0,8,16,32,64} --busbw ${SHADOW_BUSBW:-350} --out "$out/shadow.jsonl" ${SHADOW_ZERO1:+--zero1}
    ;;
  *) echo "unknown mode $mode"; exit 2 ;;
esac
echo "[gpu_suite] done"
