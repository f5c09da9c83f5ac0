#!/bin/bash
# r3 lean-run A/B on one box: lean-only kernels vs lean inside the generic kernel, operand prefetch
# (historical: the MCG_LEAN_* setup knobs these runs set were removed once the defaults were chosen;
#  the results are in profiles/r3/lean/)
# depth of the lean-only 2-D passes (MCG_LEAN_DEPTH), 2-D and 3-D.  One JSON line per run.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3ab}
mkdir -p $O
shift
b() {  # tag, env..., -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 240 python bench.py "$@" > $O/$tag.json 2>> $O/err.txt || return 1
}
for step in "$@"; do
  case $step in
    d2) b d2 MCG_LEAN_DEPTH=0 -- || exit 1 ;;
    d3) b d3 MCG_LEAN_DEPTH=3 -- || exit 1 ;;
    d4) b d4 MCG_LEAN_DEPTH=4 -- || exit 1 ;;
    mixed) b mixed MCG_LEAN_ONLY=0 -- || exit 1 ;;
    t3) b t3 MCG_LEAN_DEPTH=0 -- --problem poisson3d --grid 512 || exit 1 ;;
    t3mixed) b t3mixed MCG_LEAN_ONLY=0 -- --problem poisson3d --grid 512 || exit 1 ;;
    t3kw8) b t3kw8 MCG_LEAN_DEPTH=0 -- --problem poisson3d --grid 512 --set carry3_kw=8 || exit 1 ;;
    g4096) b g4096 MCG_LEAN_DEPTH=0 -- --grid 4096 --steps 2000 --warmup 100 || exit 1 ;;
    g4096d3) b g4096d3 MCG_LEAN_DEPTH=3 -- --grid 4096 --steps 2000 --warmup 100 || exit 1 ;;
    sim8) b sim8 MCG_LEAN_DEPTH=0 -- --sim-world 8 --sim-rank 3 --steps 400 --warmup 40 || exit 1 ;;
  esac
done
echo done
