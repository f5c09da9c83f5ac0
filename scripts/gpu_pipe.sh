#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 1100 python -m pytest tests -m gpu -x -q
step sweep 900 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg sellc8:p5:r1:P0 sellc8:p5:r1:P1 sellc8:p6:r1:P1 sell16:p5:r1:P0 sell16:p5:r1:P1
step sweep3d 900 python bench/sweep.py --problem poisson3d --n 512 --steps 40 --rounds 2 --cfg sellc8:p7:r1:P0 sellc8:p7:r1:P1
