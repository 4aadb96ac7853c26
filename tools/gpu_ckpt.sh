#!/bin/bash
# Training checkpoints on one MI355X: GPU test, then Llama-3.2-1B-shaped training with and without
# an async save inside the timed steps, and a resume from that save.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
df -h /tmp > gpurun_out/ckpt_env.log; free -g >> gpurun_out/ckpt_env.log
CK=/tmp/gtk_ckpt_$$
T="python -m gpu_topology_on_k8s_amd.models.train --model llama3-1b --batch 4 --seq 4096"
step pytest_ckpt 300 python -u -m pytest tests/test_checkpoint.py -m gpu -x -v --timeout 120 --timeout-method thread
step train_1b_base 300 $T --steps 24 --warmup 2
step train_1b_ckpt 400 $T --steps 24 --warmup 2 --save-dir $CK --save-every 12 --keep 1
step train_1b_resume 300 $T --steps 2 --warmup 0 --resume $CK
ls -la $CK $CK/* >> gpurun_out/ckpt_env.log 2>&1
rm -rf $CK
echo "== done"
