#!/bin/bash
# r3: lean-only kernels vs the generic ones, 2-D grid / waves and 3-D per-parity, one box, interleaved
# (historical: the MCG_LEAN_* setup knobs these runs set were removed once the defaults were chosen;
#  the results are in profiles/r3/lean/)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3ab2}
mkdir -p $O
b() {  # tag, env..., -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 240 python bench.py "$@" > $O/$tag.json 2>> $O/err.txt || return 1
}
for rep in 1 2; do
  b d_$rep MCG_LEAN_DEPTH=0 -- || exit 1
  b gen_$rep MCG_LEAN_ONLY=0 -- || exit 1
  b w5r2_$rep MCG_LEAN_WAVES=5 MCG_LEAN_ROUNDS=2 -- || exit 1
  b r4_$rep MCG_LEAN_ROUNDS=4 -- || exit 1
  b t3_$rep MCG_LEAN3=3 -- --problem poisson3d --grid 512 || exit 1
  b t3gen_$rep MCG_LEAN_ONLY=0 -- --problem poisson3d --grid 512 || exit 1
  b t3e_$rep MCG_LEAN3=1 -- --problem poisson3d --grid 512 || exit 1
done
echo done
