#!/bin/bash
# 3-D lean plane carry: waves per block (carry3_kw) A/B at 512^3, interleaved repeats
set -o pipefail
out=gpurun_out/${1:-kwab}
mkdir -p $out
for rep in 1 2; do
  for kw in 16 8 4; do
    timeout -k 10 300 python -u bench.py --problem poisson3d --grid 512 --steps 64 --warmup 8 --set carry3_kw=$kw \
      > $out/kw${kw}_$rep.json 2>> $out/err.log || exit 1
  done
done
