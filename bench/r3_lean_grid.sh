#!/bin/bash
# r3: lean-only 2-D grid for the latency-sized shares (4096^2, a P = 8 rank's share of 16384^2)
# (historical: the MCG_LEAN_* setup knobs these runs set were removed once the defaults were chosen;
#  the results are in profiles/r3/lean/)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3grid}
mkdir -p $O
for rep in 1 2; do
  for r in 0 1 2; do
    MCG_LEAN_ROUNDS=$r timeout -k 10 200 python bench.py --grid 4096 --steps 2000 --warmup 100 > $O/g4096_r${r}_$rep.json 2>> $O/err.txt || exit 1
    MCG_LEAN_ROUNDS=$r timeout -k 10 200 python bench.py --sim-world 8 --sim-rank 3 --steps 400 --warmup 40 > $O/sim8_r${r}_$rep.json 2>> $O/err.txt || exit 1
  done
done
echo done
