#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 900 python -m pytest tests -m gpu -x -q -k "sellc8 or dictionary or single_reduction"
step sweep2d 600 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg \
  sellc8:p5:r1 sellc8:p6:r1 sellc8:p5:r1:b32 sellc8:p5:r1:b64 sellc8:p5:r0 sell16:p5:r1 sell16:p6:r1
step sweep3d 600 python bench/sweep.py --problem poisson3d --n 512 --steps 40 --rounds 2 --cfg \
  sellc8:p7:r1 sellc8:p8:r1 sell:p7:r1 sell:p8:r1
step bench 600 python bench.py --format sellc8
