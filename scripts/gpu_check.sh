#!/bin/bash
# GPU-box check: each GPU step under its own time limit; stop at the first failing step
# (a failed test may be a device fault: nothing more runs on the GPU in this call).
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
