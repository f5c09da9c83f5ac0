#!/bin/bash
# One-GPU rows of README's headline table on the current tree (each step under its own limit).
set -o pipefail
out=gpurun_out/readme
mkdir -p $out
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 150 python bench.py "$@" > $out/$name.json 2> $out/$name.err || return 1
  tail -1 $out/$name.json
}
run p2d_default &&
run p2d_dia0 --set carry_dia=0 &&
run p2d_store --set ap_recompute=0 &&
run p2d_generic --set carry=0 &&
run p2d_pipelined --recurrence 2 &&
run p4096_default --grid 4096 --steps 2000 --warmup 200 &&
run p3d_default --problem poisson3d --grid 512 &&
run p3d_store --problem poisson3d --grid 512 --set ap_recompute=0
