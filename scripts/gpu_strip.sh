#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step sweep 900 python bench/sweep.py --n 16384 --steps 40 --rounds 3 --cfg sellc8:p5:r1:S0 sellc8:p5:r1 sellc8:p5:r1:P0 sell16:p5:r1:S0 sell16:p5:r1
step pmc 600 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum --kernel-trace --output-format csv -d gpurun_out/p4_strip -o run -- python bench.py --steps 4 --warmup 2 --no-verify --phases 0
step tests 1100 python -m pytest tests -m gpu -x -q
step sweep4k 900 python bench/sweep.py --n 4096 --steps 400 --warmup 20 --rounds 3 --cfg sellc8:p5:r1:S0 sellc8:p5:r1
