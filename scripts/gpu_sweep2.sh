#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step sweep 900 python bench/sweep.py --n 16384 --steps 30 --rounds 2 --cfg \
  csr:v1:p6:b8:u2 csr:v1:p8:b8:u2 csr:v1:p6:b4:u2 csr:v1:p6:b16:u2 \
  csr:v0:p6:b6:u2 csr:v0:p8:b6:u2 csr:v0:p6:b4:u2 \
  csr:v2:p8:b8:u2 csr:v2:p4:b8:u2 csr:v2:p8:b16:u2 \
  sell:v1:p6:b8:u2 sell:v1:p8:b8:u2 sell:v1:p6:b16:u2 sell:v1:p6:b4:u2 \
  csr:v1:p6:b8:u1 csr:v1:p6:b8:u4
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify
