#!/bin/bash
# r3: 3-D lean runs per pass parity (MCG_LEAN3: bit 0 even, bit 1 odd passes), 512^3, interleaved
# (historical: the MCG_LEAN_* setup knobs these runs set were removed once the defaults were chosen;
#  the results are in profiles/r3/lean/)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3l3}
mkdir -p $O
for rep in 1 2; do
  for m in 3 1 0 2; do
    MCG_LEAN3=$m timeout -k 10 200 python bench.py --problem poisson3d --grid 512 > $O/l3_${m}_$rep.json 2>> $O/err.txt || exit 1
  done
done
echo done
