#!/bin/bash
# interleaved {r, Ap} pairs: GPU tests touching the single-reduction path, then a sweep
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 900 python -m pytest tests -m gpu -x -q -k "interleave or single_reduction or local_ranks or checkpoint or fault or serialised"
step sweep 600 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg \
  sell16:p6:r0 sell16:p6:r1:i0 sell16:p6:r1:i1 sell16:p8:r1:i1 sell16:p4:r1:i1
