#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 1100 python -m pytest tests -m gpu -x -q
step sweep 600 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg sellc8:p5:r1 sell16:p5:r1 sellc8:p5:r0
step bench 600 python bench.py
step rs 900 python bench.py --problem randspd --rows 4000000 --band 4096 --density 0.16 --steps 30 --warmup 4
