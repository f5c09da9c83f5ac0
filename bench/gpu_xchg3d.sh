# 3-D plane carry, block exchange (carry_3d=2) vs gathers (carry_3d=1): tests, benches, counters
# usage: bash bench/gpu_xchg3d.sh [sweep]
set -o pipefail
cd $GRAFT_REPO_ROOT
if [ "$1" = "place" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_place.log 2>&1 || { tail -30 gpurun_out/pytest_place.log; exit 1; }
  tail -1 gpurun_out/pytest_place.log
  for rep in 1 2 3 4 5; do
    for t in 3 1; do
      timeout -k 10 200 python bench.py --problem poisson3d --grid 512 --phases 0 --set placement_tries=$t > gpurun_out/x.json 2>/dev/null || exit 1
      echo "3d tries=$t $(python3 -c "import json; d=json.load(open('gpurun_out/x.json')); print(d['value'], d['check']['placement_gain'], d['check']['setup_s'])")" >> gpurun_out/place.log
      timeout -k 10 200 python bench.py --phases 0 --set placement_tries=$t > gpurun_out/x.json 2>/dev/null || exit 1
      echo "2d tries=$t $(python3 -c "import json; d=json.load(open('gpurun_out/x.json')); print(d['value'], d['check']['placement_gain'], d['check']['setup_s'])")" >> gpurun_out/place.log
    done
  done
  exit 0
fi
if [ "$1" = "cfg" ]; then
  # usage: bash bench/gpu_xchg3d.sh cfg REPS "args A" "args B" ...   (bench.py args per config)
  reps=$2; shift 2
  for rep in $(seq $reps); do
    for c in "$@"; do
      timeout -k 10 200 python bench.py --phases 0 $c > gpurun_out/x.json 2>/dev/null || exit 1
      echo "$c | $(python3 -c "import json; d=json.load(open('gpurun_out/x.json')); print(d['value'], d['check']['placement_gain'], d['check'].get('placement_lead_trial'), d['check']['setup_s'])")" >> gpurun_out/cfg.log
    done
  done
  exit 0
fi
if [ "$1" = "skew" ]; then
  for rep in 1 2 3 4; do
    for k in 0 1 7; do
      timeout -k 10 200 python bench.py --problem poisson3d --grid 512 --phases 0 --set vec_skew=$k > gpurun_out/x.json 2>/dev/null || exit 1
      echo "3d skew=$k $(python3 -c "import json; print(json.load(open('gpurun_out/x.json'))['value'])")" >> gpurun_out/skew.log
    done
  done
  for rep in 1 2 3; do
    for k in 0 1; do
      timeout -k 10 200 python bench.py --phases 0 --set vec_skew=$k > gpurun_out/x.json 2>/dev/null || exit 1
      echo "2d skew=$k $(python3 -c "import json; print(json.load(open('gpurun_out/x.json'))['value'])")" >> gpurun_out/skew.log
    done
  done
  exit 0
fi
if [ "$1" = "sweep" ]; then
  for rep in 1 2; do
    for s in "carry_3d=2 carry_depth=1" "carry_3d=2 carry_depth=2" "carry_3d=2 carry_depth=3" "carry_3d=1 carry_depth=1"; do
      a=""; for kv in $s; do a="$a --set $kv"; done
      timeout -k 10 200 python bench.py --problem poisson3d --grid 512 --phases 0 $a > gpurun_out/x.json 2>/dev/null || exit 1
      echo "$s $(python3 -c "import json; print(json.load(open('gpurun_out/x.json'))['value'])")" >> gpurun_out/xchg3d_sweep.log
    done
  done
  exit 0
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "carry" > gpurun_out/pytest_xchg.log 2>&1 || { tail -30 gpurun_out/pytest_xchg.log; exit 1; }
tail -2 gpurun_out/pytest_xchg.log
for m in 2 1 2 1; do
  timeout -k 10 200 python bench.py --problem poisson3d --grid 512 --set carry_3d=$m >> gpurun_out/xchg3d.jsonl 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE -d gpurun_out/pmcx_a -o run -- python3 bench.py --problem poisson3d --grid 512 --steps 4 --warmup 2 --phases 0 --no-verify > gpurun_out/pmcx_a.log 2>&1
