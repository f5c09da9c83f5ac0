# round check + 4096^2 bench (graph_iters default)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash bench/gpu_round_check.sh || exit 1
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 150 python bench.py --grid 4096 > gpurun_out/b4096.json 2>/dev/null || exit 1
for f in bench_check bench_check3d b4096; do python -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['check']['ok'],flush=True)"; done
