#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step bench_default 600 python bench.py
step bench_csr 600 python bench.py --format csr --steps 100
step bench_f1 600 python bench.py --recurrence 1 --steps 100
step bench_4096 600 python bench.py --grid 4096 --steps 500
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 5 --warmup 1 --no-verify
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 5 --warmup 1 --no-verify
