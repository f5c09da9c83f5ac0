# iterations per hipGraph launch: pairs (2) vs 8 vs 32, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_gi.log 2>&1 || { tail -30 gpurun_out/pt_gi.log; exit 1; }
tail -1 gpurun_out/pt_gi.log
for rep in 1 2; do
  for grid in 4096 16384; do
    for gi in 2 8 32; do
      timeout -k 10 150 python bench.py --grid $grid --phases 0 --set graph_iters=$gi > gpurun_out/gi.json 2>gpurun_out/gi.err || { tail -5 gpurun_out/gi.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/gi.json'));print('grid $grid graph_iters=$gi',d['value'],d['check']['ok'],flush=True)" | tee -a gpurun_out/graph_iters.log
    done
  done
done
