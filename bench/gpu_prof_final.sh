# Kernel stats of the default 2-D and 3-D bench paths (placement probe on), one GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pf2d -o run --output-format csv -- python3 bench.py --steps 20 --warmup 4 --phases 0 > gpurun_out/pf2d.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pf3d -o run --output-format csv -- python3 bench.py --problem poisson3d --grid 512 --steps 20 --warmup 4 --phases 0 > gpurun_out/pf3d.log 2>&1 || exit 1
