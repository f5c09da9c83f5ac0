#!/bin/bash
# Halo ahead on the side stream next to the all-reduce (overlap 1, dual communicators) vs everything
# in one stream order (overlap 0, what single-communicator mode runs), DelayComm D = 10 / H = 10 us,
# interleaved repeats.
set -o pipefail
out=gpurun_out/ovab
mkdir -p $out
for rep in 1 2 3; do
  for g in 16384 4096; do
    timeout -k 10 200 python bench/pipe_latency.py --grid $g --world 8 --rank 3 --recurrences 1 --graphs 1 --overlaps 1,0 --delays 10 --halo-us 10 --iters 640 >> $out/ab.jsonl 2>> $out/err.log || exit 1
  done
  timeout -k 10 200 python bench/pipe_latency.py --problem poisson3d --grid 512 --world 8 --rank 3 --recurrences 1 --graphs 1 --overlaps 1,0 --delays 10 --halo-us 10 --iters 640 >> $out/ab.jsonl 2>> $out/err.log || exit 1
done
