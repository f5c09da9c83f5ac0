# Round-end style check on one GPU: GPU tests, smoke(), headline bench, 3-D bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py > gpurun_out/bench_check.json 2>gpurun_out/bench_check.err || exit 1
timeout -k 10 200 python bench.py --problem poisson3d --grid 512 > gpurun_out/bench_check3d.json 2>/dev/null || exit 1
