#!/bin/bash
# irregular-sparsity path (BASELINE.json config 5, scaled to one GPU): random SPD, ~1300 nnz/row
source scripts/gpu_check.sh
export TMPDIR=/tmp
R="--problem randspd --rows 4000000 --band 4096 --density 0.16 --steps 30 --warmup 4"
step rs_sell16 900 python bench.py $R --format sell16
step rs_csr 900 python bench.py $R --format csr
step rs_csr_r0 900 python bench.py $R --format csr --recurrence 0
step rs_sell16_r0 900 python bench.py $R --format sell16 --recurrence 0
