#!/bin/bash
# SELL-64/c8 dictionary format: GPU tests, then sweeps on 2D / 3D Poisson
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 900 python -m pytest tests -m gpu -x -q -k "sellc8 or dictionary or interleave or single_reduction"
step sweep2d 600 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg \
  sell16:p6:r1 sellc8:p6:r1 sellc8:p8:r1 sellc8:p4:r1 sellc8:p8:r1:b32 sellc8:p6:r0 sellc8:p8:r0
step sweep3d 600 python bench/sweep.py --problem poisson3d --n 512 --steps 40 --rounds 2 --cfg \
  sell:p6:r1 sellc8:p6:r1 sellc8:p8:r1
step bench 600 python bench.py --format sellc8
