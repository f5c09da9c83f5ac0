# r3: DRAM / L2 counters of the scrambled config-5 share, tiles vs CSR split pass, + tiles GPU tests
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_irregular.py -x -q --timeout 240 --timeout-method thread -k tiles > gpurun_out/r3_tiles_tests.log 2>&1 || { tail -30 gpurun_out/r3_tiles_tests.log; exit 1; }
tail -1 gpurun_out/r3_tiles_tests.log
S="--problem randspd --rows 100000000 --band 410 --density 1.0 --scramble 1 --sim-world 8 --sim-rank 3 --phases 0 --no-verify"
timeout -k 10 300 python bench.py $S --steps 10 --warmup 3 > gpurun_out/r3_c5scr_tiles2.json 2>/dev/null || exit 1
tail -c 200 gpurun_out/r3_c5scr_tiles2.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE -d gpurun_out/r3_pmc_c5t_dram -o p --output-format csv -- python3 bench.py $S --steps 2 --warmup 1 > /dev/null 2> gpurun_out/r3_pmc_c5t_dram.err || exit 1
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/r3_pmc_c5t_l2 -o p --output-format csv -- python3 bench.py $S --steps 2 --warmup 1 > /dev/null 2> gpurun_out/r3_pmc_c5t_l2.err || exit 1
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE -d gpurun_out/r3_pmc_c5c_dram -o p --output-format csv -- python3 bench.py $S --steps 2 --warmup 1 --format csr --set tiles=0 > /dev/null 2> gpurun_out/r3_pmc_c5c_dram.err || exit 1
python bench/pmc_csv.py gpurun_out/r3_pmc_c5t_dram k_tiles
python bench/pmc_csv.py gpurun_out/r3_pmc_c5t_l2 k_tiles
python bench/pmc_csv.py gpurun_out/r3_pmc_c5c_dram k_split_spmv
