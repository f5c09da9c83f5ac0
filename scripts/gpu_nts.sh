#!/bin/bash
# A/B: plain vs non-temporal vector stores in the single-reduction pass (rebuilds on the box)
source scripts/gpu_check.sh
export TMPDIR=/tmp
step base 600 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg sellc8:p5:r1
step rebuild 900 make -j16 EXTRA_HIPFLAGS=-DMCG_NT_STORES=1 -B build/gpu/cg_fused1.o all
step nts 600 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg sellc8:p5:r1
