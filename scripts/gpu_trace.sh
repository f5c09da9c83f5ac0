#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
export MCG_TRACE=1
step trace 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- python bench.py --grid 4096 --steps 10 --warmup 2 --no-verify
