#!/bin/bash
# r3 lean-run profiles: kernel stats and DRAM counters per pass of the default 2-D path (16384^2),
# plus the GPU suite.  Each step under its own limit; the first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3l}
mkdir -p $O
run_stats() {  # tag, bench args
  local tag=$1; shift
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o p -- python3 $R/bench.py --phases 0 "$@" > $O/$tag.json 2> $O/$tag.err) || return 1
  f=$(find $O/$tag -name "*kernel_stats.csv" | head -1)
  python3 $R/bench/prof_summary.py --stats $f --title "$tag: bench.py $*" > $O/$tag.md || return 1
}
run_dram() {  # tag, kernel substring, bench args
  local tag=$1 k=$2; shift 2
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE -d $O/$tag -o p --output-format csv -- python3 $R/bench.py --phases 0 "$@" > /dev/null 2> $O/$tag.err) || return 1
  python3 $R/bench/pmc_csv.py $O/$tag $k > $O/$tag.txt || return 1
}
shift
for step in "$@"; do
  case $step in
    stats2d) run_stats stats_16384 --steps 64 --warmup 8 || exit 1 ;;
    stats3d) run_stats stats_512 --problem poisson3d --grid 512 --steps 64 --warmup 8 || exit 1 ;;
    dram2d) run_dram dram_16384 k_cg_carry_ar --steps 8 --warmup 2 || exit 1 ;;
    dram3d) run_dram dram_512 k_cg_carry_ar3 --problem poisson3d --grid 512 --steps 8 --warmup 2 || exit 1 ;;
    sq2d) (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d $O/sq_16384 -o p --output-format csv -- python3 $R/bench.py --phases 0 --steps 8 --warmup 2 > /dev/null 2> $O/sq_16384.err) && python3 $R/bench/pmc_csv.py $O/sq_16384 k_cg_carry_ar > $O/sq_16384.txt || exit 1 ;;
    sq3d) (cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU -d $O/sq_512 -o p --output-format csv -- python3 $R/bench.py --phases 0 --problem poisson3d --grid 512 --steps 8 --warmup 2 > /dev/null 2> $O/sq_512.err) && python3 $R/bench/pmc_csv.py $O/sq_512 k_cg_carry_ar3 > $O/sq_512.txt || exit 1 ;;
    suite) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1 ;;
    b4096) timeout -k 10 200 python bench.py --grid 4096 --steps 2000 --warmup 100 > $O/bench_4096.json 2>> $O/bench.err || exit 1 ;;
    b3d) timeout -k 10 200 python bench.py --problem poisson3d --grid 512 > $O/bench_512.json 2>> $O/bench.err || exit 1 ;;
    bsim8) timeout -k 10 200 python bench.py --sim-world 8 --sim-rank 3 --steps 400 --warmup 40 > $O/bench_sim8.json 2>> $O/bench.err || exit 1 ;;
    bench) timeout -k 10 200 python bench.py > $O/bench.json 2>> $O/bench.err || exit 1 ;;
  esac
done
echo done
