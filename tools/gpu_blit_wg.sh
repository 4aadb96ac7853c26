#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step blit_default 120 python tools/blit_wg_probe.py
for wg in 16 64 256 1024 4096; do
  DEBUG_CLR_LIMIT_BLIT_WG=$wg step blit_wg_$wg 120 python tools/blit_wg_probe.py
done
echo "== done"
