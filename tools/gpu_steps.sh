#!/bin/bash
# Helper sourced by gpurun commands: run one GPU step under its own time limit, log to
# gpurun_out/<name>.log, and stop the whole call on a timeout/abort/segfault (rc >= 124).
mkdir -p gpurun_out
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name (limit ${secs}s): $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "== stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
