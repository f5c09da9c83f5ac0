# placement probe depth: default (3 sets x 4 leads) vs deeper probes, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for cfg in "3 4" "4 8" "3 8" "8 8"; do
    set -- $cfg
    timeout -k 10 150 python bench.py --steps 200 --warmup 20 --phases 0 --set placement_tries=$1 --set placement_leads=$2 > gpurun_out/ps.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ps.json'));c=d['check'];print('2d tries=$1 leads=$2',d['value'],c.get('placement_gain'),c.get('setup_s'),flush=True)" | tee -a gpurun_out/place_sweep.log
  done
done
