#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step pytest_aux 900 python -m pytest tests/test_gpu_aux.py -x -q
step pytest_gpu 900 python -m pytest tests -m gpu -q
step trace 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- python bench.py --grid 4096 --steps 10 --warmup 2 --no-verify
