# default placement probe after a change: GPU solver tests + 3 headline + 1 3-D bench
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_pc.log 2>&1 || { tail -30 gpurun_out/pt_pc.log; exit 1; }
tail -1 gpurun_out/pt_pc.log
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py > gpurun_out/pc2d_$rep.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/pc2d_$rep.json'));c=d['check'];print('2d',d['value'],c.get('placement_gain'),c.get('setup_s'),flush=True)"
done
timeout -k 10 150 python bench.py --problem poisson3d --grid 512 > gpurun_out/pc3d.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/pc3d.json'));c=d['check'];print('3d',d['value'],c.get('placement_gain'),c.get('setup_s'),flush=True)"
