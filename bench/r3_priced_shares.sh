#!/bin/bash
# Per-rank shares priced with a collective latency: rank 3 (rank 1 at P = 2) of a P-rank run on one
# GPU, the single-reduction default path, each all-reduce a device-side delay D and each halo H
# (DelayComm), hipGraphs on.  us per iteration -> projected whole-job it/s = 1e6 / us.
set -o pipefail
out=gpurun_out/priced
mkdir -p $out
for g in 16384 4096; do
  for w in 2 4 8; do
    r=$(( w > 2 ? 3 : 1 ))
    timeout -k 10 200 python bench/pipe_latency.py --grid $g --world $w --rank $r --recurrences 1 --graphs 1 --overlaps 1,0 --delays 0,10,20 --halo-us 10 --iters 320 >> $out/shares.jsonl 2> $out/err_${g}_$w.log || exit 1
  done
done
for w in 2 4 8; do
  r=$(( w > 2 ? 3 : 1 ))
  timeout -k 10 200 python bench/pipe_latency.py --problem poisson3d --grid 512 --world $w --rank $r --recurrences 1 --graphs 1 --delays 0,10,20 --halo-us 10 --iters 320 >> $out/shares.jsonl 2> $out/err_512_$w.log || exit 1
done
grep -c . $out/shares.jsonl
