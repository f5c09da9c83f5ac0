#!/bin/bash
# refreshed evidence for the default bench path: kernel stats, DRAM-level bytes, bench lines
source scripts/gpu_check.sh
export TMPDIR=/tmp
step bench 600 python bench.py
step bench3d 600 python bench.py --problem poisson3d --grid 512
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python bench.py --steps 20 --warmup 2 --no-verify --phases 0
step pmc_dram 600 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum --kernel-trace --output-format csv -d gpurun_out/pmc_final_dram -o run -- python bench.py --steps 4 --warmup 2 --no-verify --phases 0
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_final_fetch -o run -- python bench.py --steps 4 --warmup 2 --no-verify --phases 0
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_final_write -o run -- python bench.py --steps 4 --warmup 2 --no-verify --phases 0
