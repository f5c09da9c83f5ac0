# kernel-trace of 4096^2 with pair graphs vs 32-iteration graphs: inter-kernel gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for gi in 2 32; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/gap$gi -o run --output-format csv -- python3 bench.py --grid 4096 --steps 128 --warmup 4 --phases 0 --set graph_iters=$gi > gpurun_out/gap$gi.log 2>&1 || exit 1
done
