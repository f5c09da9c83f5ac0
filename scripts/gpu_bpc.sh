#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step sweep 900 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg sellc8:p5:r1 sellc8:p5:r1:b8 sellc8:p5:r1:b12 sellc8:p5:r1:b16 sellc8:p5:r1:b24 sellc8:p5:r1:b32
step sweep4k 900 python bench/sweep.py --n 4096 --steps 400 --warmup 20 --rounds 3 --cfg sellc8:p5:r1 sellc8:p5:r1:b8 sellc8:p5:r1:b16 sellc8:p5:r1:b24
