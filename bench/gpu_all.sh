set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 200 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --phases 0 > gpurun_out/prof_final.log 2>&1 || exit 1
