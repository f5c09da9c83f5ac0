#!/bin/bash
# DRAM-level traffic + unit-busy counters of the default bench path (PMC runs: --kernel-trace only)
source scripts/gpu_check.sh
export TMPDIR=/tmp
B="python bench.py --steps 6 --warmup 2 --no-verify --phases 0"
step pmc_dram 600 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum --kernel-trace --output-format csv -d gpurun_out/pmc_dram -o run -- $B
step pmc_busy 600 rocprofv3 --pmc TA_BUSY_avr MemUnitStalled --kernel-trace --output-format csv -d gpurun_out/pmc_busy -o run -- $B
step pmc_gmi 600 rocprofv3 --pmc TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_IO_32B_sum --kernel-trace --output-format csv -d gpurun_out/pmc_gmi -o run -- $B
step pmc_wait 600 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_wait -o run -- $B
