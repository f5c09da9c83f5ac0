#!/bin/bash
# r3: repeats of the latency-sized benches (4096^2, a P = 8 rank's share of 16384^2) on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3rep}
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --grid 4096 --steps 2000 --warmup 100 > $O/g4096_$rep.json 2>> $O/err.txt || exit 1
  timeout -k 10 200 python bench.py --sim-world 8 --sim-rank 3 --steps 400 --warmup 40 > $O/sim8_$rep.json 2>> $O/err.txt || exit 1
done
echo done
