# r2 check: new fused-reduce tests, full GPU suite, benches (inline + spawn route), 4096^2 kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_reduce.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || { tail -60 gpurun_out/pytest_fused.log; exit 1; }
tail -3 gpurun_out/pytest_fused.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py > gpurun_out/b16k.json 2>gpurun_out/b16k.err || { cat gpurun_out/b16k.err; exit 1; }
timeout -k 10 200 python bench.py --gpus 1 --spawn > gpurun_out/b16k_spawn.json 2>gpurun_out/b16k_spawn.err || { cat gpurun_out/b16k_spawn.err; exit 1; }
timeout -k 10 200 python bench.py --force-comm > gpurun_out/b16k_fc.json 2>gpurun_out/b16k_fc.err || { cat gpurun_out/b16k_fc.err; exit 1; }
timeout -k 10 200 python bench.py --set fused_reduce=0 > gpurun_out/b16k_nofr.json 2>gpurun_out/b16k_nofr.err || exit 1
timeout -k 10 200 python bench.py --grid 4096 --steps 2000 --warmup 100 > gpurun_out/b4096.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --grid 4096 --steps 2000 --warmup 100 --set fused_reduce=0 > gpurun_out/b4096_nofr.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --problem poisson3d --grid 512 > gpurun_out/b512.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --problem poisson3d --grid 512 --set fused_reduce=0 > gpurun_out/b512_nofr.json 2>/dev/null || exit 1
python bench.py --gpus 2 > gpurun_out/b_gpus2.out 2> gpurun_out/b_gpus2.err; echo "gpus2 rc=$?" >> gpurun_out/b_gpus2.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4096fc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --grid 4096 --steps 64 --warmup 8 --phases 0 --force-comm > $GRAFT_REPO_ROOT/gpurun_out/prof4096fc.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof4096fc.log; exit 1; }
echo ALLDONE
