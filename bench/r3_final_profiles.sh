#!/bin/bash
# r3 end-of-round profiles of the default paths: kernel stats (16384^2, 512^3, the pipelined form at
# a P = 8 share of 4096^2) and DRAM counters per pass (16384^2, 512^3).  Each step under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3f
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run_stats() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o p -- python3 $R/bench.py --phases 0 "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  f=$(find $O/$tag -name "*kernel_stats.csv" | head -1)
  python3 $R/bench/prof_summary.py --stats $f --title "$tag: bench.py $*" > $O/$tag.md || return 1
}
run_dram() {  # tag, kernel substring, bench args
  local tag=$1 k=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE -d $O/$tag -o p --output-format csv -- python3 $R/bench.py --phases 0 "$@" > /dev/null 2> $O/$tag.err || return 1
  python3 $R/bench/pmc_csv.py $O/$tag $k > $O/$tag.txt || return 1
}
run_stats stats_16384 --steps 64 --warmup 8 &&
run_stats stats_512 --problem poisson3d --grid 512 --steps 64 --warmup 8 &&
run_stats stats_pipe_4096_p8 --grid 4096 --recurrence 2 --sim-world 8 --sim-rank 3 --steps 256 --warmup 32 &&
run_dram dram_16384 k_cg_carry_ar --steps 8 --warmup 2 &&
run_dram dram_512 k_cg_carry_ar3 --problem poisson3d --grid 512 --steps 8 --warmup 2 &&
echo done
