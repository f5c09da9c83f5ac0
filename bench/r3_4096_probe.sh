#!/bin/bash
# 4096^2: where the even pass's time goes -- kernel stats with the in-kernel reduction off
# (fused_reduce=0: a separate reduce launch) and with the generic (non-lean) kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-p4096}
mkdir -p $O
for v in "fr0 fused_reduce=0" "gen dia_uniform=0"; do
  set -- $v
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1 -o p -- python3 $R/bench.py --grid 4096 --steps 640 --warmup 64 --phases 0 --set $2 > $O/$1.json 2> $O/$1.err) || exit 1
  f=$(find $O/$1 -name "*kernel_stats.csv" | head -1)
  python3 $R/bench/prof_summary.py --stats $f --title "4096^2 --set $2" > $O/$1.md || exit 1
done
