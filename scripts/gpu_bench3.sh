#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step bench_default 600 python bench.py
step bench_classic 600 python bench.py --recurrence 0
step bench_3d 600 python bench.py --problem poisson3d --grid 512
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ra -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify
