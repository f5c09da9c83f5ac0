#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step sweep 1000 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg \
  sell16:p6:b16 sell16:p6:b32 sell16:p6:b24 sell16:p6:b32:B4:u1 sell16:p6:b32:B8:u1 sell16:p6:b32:B4:u2 sell16:p6:b32:B16:u1 sell16:p6:b48:B4:u1 sell16:p8:b32:B4:u1
