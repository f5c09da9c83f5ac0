#!/bin/bash
# Placement probe depth (placement_tries allocations x placement_leads start offsets), interleaved
# bench runs on one box: 2-D 16384^2 and 3-D 512^3.
set -o pipefail
out=gpurun_out/ptries
mkdir -p $out
one() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 150 python bench.py --phases 0 "$@" > $out/$tag.json 2> $out/$tag.err || return 1
  python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); c=d['check']; print('$tag', round(d['value'],1), c.get('placement_gain'), c.get('setup_s'))"
}
for rep in 1 2; do
  one 2d_t3_$rep --set placement_tries=3 &&
  one 2d_t6_$rep --set placement_tries=6 &&
  one 2d_t6l16_$rep --set placement_tries=6 --set placement_leads=16 &&
  one 3d_t3_$rep --problem poisson3d --grid 512 --set placement_tries=3 &&
  one 3d_t6_$rep --problem poisson3d --grid 512 --set placement_tries=6 || exit 1
done
