set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py > gpurun_out/bench_final2d.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --problem poisson3d --grid 512 > gpurun_out/bench_final3d.json 2>/dev/null || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3d -o run --output-format csv -- python3 bench.py --problem poisson3d --grid 512 --steps 20 --warmup 4 --phases 0 > gpurun_out/prof3d.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2d -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --phases 0 > gpurun_out/prof2d.log 2>&1 || exit 1
bash bench/pmc_3d.sh
