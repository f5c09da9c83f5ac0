# rocprofv3 counter passes of the 16384^2 bench pass, generic vs line-carry (one pass per counter set)
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for c in ${CARRY_SET:-0 1}; do
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_c${c}_a -o run -- python3 bench.py --steps 4 --warmup 2 --phases 0 --no-verify --set carry=$c > gpurun_out/pmc_c${c}_a.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES -d gpurun_out/pmc_c${c}_b -o run -- python3 bench.py --steps 4 --warmup 2 --phases 0 --no-verify --set carry=$c > gpurun_out/pmc_c${c}_b.log 2>&1
done
