#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step sweep 600 python bench/sweep.py --n 16384 --steps 30 --formats csr sell --bpc 2 4 6 8 16 --rounds 2
step prof_csr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_csr -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify
step prof_sell 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sell -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify --format sell
