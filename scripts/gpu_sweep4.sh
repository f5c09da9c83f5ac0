#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step membw 300 ./build/membw
step sweep 1000 python bench/sweep.py --n 16384 --steps 30 --rounds 3 --cfg \
  sell:p6:b16 sell:p6:b16:s2 sell:p6:b8:s2 sell:p6:b4:s2 sell:p6:b32 csr:v1:p6:b4 sell:p8:b16:s2
