#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step sweep 1000 python bench/sweep.py --n 16384 --steps 30 --rounds 3 --cfg \
  sell:p6:b16 sell:p6:b16:r1 sell:p6:b8:r1 sell:p6:b8:s2:r1 sell:p6:b4:s2:r1 csr:v1:p6:b4:r1 csr:v1:p6:b8:r1
