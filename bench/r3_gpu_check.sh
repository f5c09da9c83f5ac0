# r3 GPU check after a change: full GPU suite + smoke + default bench (16384^2) + 512^3
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
timeout -k 10 200 python bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || exit 1
timeout -k 10 200 python bench.py --problem poisson3d --grid 512 > gpurun_out/r3_bench3d.json 2>> gpurun_out/r3_bench.err || exit 1
python -c "
import json
for f in ('gpurun_out/r3_bench.json', 'gpurun_out/r3_bench3d.json'):
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d['config']['pass'])"
