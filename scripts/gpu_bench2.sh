#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step bench_default 600 python bench.py
step bench_f1 600 python bench.py --recurrence 1 --steps 100
step bench_3d 600 python bench.py --problem poisson3d --grid 512 --steps 100
step sweep_f1 1000 python bench/sweep.py --n 16384 --steps 40 --rounds 2 --cfg sell16:p6:r1 sell16:p6:b32:r1 sell16:p6:b16:r1 sell16:p6:r0
