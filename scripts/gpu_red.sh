#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 1100 python -m pytest tests -m gpu -x -q
step b4096 600 python bench.py --grid 4096 --steps 2000 --warmup 100
step bench 600 python bench.py
step prof4096 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4096 -o run --output-format csv -- python bench.py --grid 4096 --steps 200 --warmup 10 --no-verify
