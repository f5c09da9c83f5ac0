#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step sweep 1000 python bench/sweep.py --n 16384 --steps 30 --rounds 3 --cfg \
  csr:v1:p6:b8 csr:v1:p6:b8:n1 csr:v1:p6:b8:x1 csr:v1:p6:b8:n1:x1 \
  csr:v1:p6:b4 csr:v1:p6:b4:n1:x1 csr:v0:p6:b6:x1 \
  sell:p6:b16 sell:p6:b16:n1 sell:p6:b16:x1 sell:p6:b16:n1:x1 sell:p6:b8:n1:x1
