#!/bin/bash
# where do the extra reads of the single-reduction pass come from? DRAM read bytes vs grid / XCD map / N
source scripts/gpu_check.sh
export TMPDIR=/tmp
P="--pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum --kernel-trace --output-format csv"
B="python bench.py --steps 4 --warmup 2 --no-verify --phases 0"
step x1 600 rocprofv3 $P -d gpurun_out/p3_x1 -o run -- $B --set xcd_map=1
step b8 600 rocprofv3 $P -d gpurun_out/p3_b8 -o run -- $B --blocks-per-cu 8
step b4 600 rocprofv3 $P -d gpurun_out/p3_b4 -o run -- $B --blocks-per-cu 4
step n4096 600 rocprofv3 $P -d gpurun_out/p3_n4096 -o run -- $B --grid 4096
step n1024 600 rocprofv3 $P -d gpurun_out/p3_n1024 -o run -- $B --grid 1024
step n16384_sell16 600 rocprofv3 $P -d gpurun_out/p3_sell16 -o run -- $B --format sell16
