cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_irregular.py -x -v --timeout 180 --timeout-method thread -k "tiles" > gpurun_out/r3_tiles_tests.log 2>&1 || { tail -30 gpurun_out/r3_tiles_tests.log; exit 1; }
tail -3 gpurun_out/r3_tiles_tests.log
