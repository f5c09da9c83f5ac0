# r3 GPU checkpoint: full GPU suite + smoke, then the scrambled config-5 share (tiles vs CSR split)
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
S="--problem randspd --rows 100000000 --band 410 --density 1.0 --scramble 1 --sim-world 8 --sim-rank 3"
timeout -k 10 400 python bench.py $S --steps 10 --warmup 3 --phases 5 > gpurun_out/r3_c5scr_tiles.json 2> gpurun_out/r3_c5scr_tiles.err || exit 1
tail -c 600 gpurun_out/r3_c5scr_tiles.json
timeout -k 10 400 python bench.py $S --steps 5 --warmup 2 --phases 0 --format csr --set tiles=0 > gpurun_out/r3_c5scr_csr.json 2> gpurun_out/r3_c5scr_csr.err || exit 1
tail -c 300 gpurun_out/r3_c5scr_csr.json
