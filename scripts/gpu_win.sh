#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 900 python -m pytest tests -m gpu -x -q -k "window or interleave or dictionary or dense_halo or local_ranks_match"
R="--problem randspd --rows 4000000 --band 4096 --density 0.16 --steps 30 --warmup 4"
step rs_win 900 python bench.py $R --format sell16
step rs_sweep 900 python bench/sweep.py --problem randspd --steps 20 --warmup 3 --rounds 1 --cfg sell16:r1:w1:p8 sell16:r1:w1:p6 sell16:r1:w1:p4 sell16:r1:w0:p8
