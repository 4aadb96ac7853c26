#!/bin/bash
# End-of-session check: whole GPU suite, smoke(), k=1 headline bench.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
source tools/gpu_steps.sh
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_k1 300 python3 bench.py --steps 50 --warmup 10
echo "== done"
