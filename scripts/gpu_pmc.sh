#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
for fmt in csr sell; do
step pmc_fetch_$fmt 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_$fmt -o run -- python bench.py --steps 5 --warmup 1 --no-verify --format $fmt
step pmc_write_$fmt 600 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_write_$fmt -o run -- python bench.py --steps 5 --warmup 1 --no-verify --format $fmt
done
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify
