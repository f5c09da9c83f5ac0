set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench/rehearse_ranks.py --problem poisson3d --n 512 --iters 30 --world 1 2 4 8 > gpurun_out/rehearse3d.log 2>&1 || exit 1
bash bench/pmc_3d.sh
