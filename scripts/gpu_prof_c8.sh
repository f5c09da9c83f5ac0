#!/bin/bash
# kernel stats + PMC (HBM bytes, L2 hit) of the default bench path (SELL-64/c8, single reduction)
source scripts/gpu_check.sh
export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c8 -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_c8 -o run -- python bench.py --steps 5 --warmup 1 --no-verify
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_write_c8 -o run -- python bench.py --steps 5 --warmup 1 --no-verify
