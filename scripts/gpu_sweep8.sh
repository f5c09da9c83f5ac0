#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step sweep2d 900 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg \
  sellc8:p5:r1 sellc8:p5:r1:x1 sellc8:p5:r1:n1 sellc8:p5:r1:b40 sellc8:p5:r1:b64 sellc8:p5:r1:b96 sellc8:p5:r1:b128 sellc8:p5:r1:g0
