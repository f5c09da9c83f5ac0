# rocprofv3 counter passes of the 512^3 bench pass (generic + XCD plane sweep, pipelined)
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc3d_a -o run -- python3 bench.py --problem poisson3d --grid 512 --steps 4 --warmup 2 --phases 0 --no-verify > gpurun_out/pmc3d_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES -d gpurun_out/pmc3d_b -o run -- python3 bench.py --problem poisson3d --grid 512 --steps 4 --warmup 2 --phases 0 --no-verify > gpurun_out/pmc3d_b.log 2>&1
