#!/bin/bash
# CU-masked compute stream vs the 270-VGPR side-stream collective (profiles/r3_cumask_probe.md).
#  probe : bench/cumask_probe.py (hog grid on a masked queue; fat / thin spin and RCCL loopback beside it)
#  split : a P = 8 rank's share, interior || halo split (halo_ahead 0) vs halo ahead vs one stream order,
#          DelayComm with the fat spin as the halo (RCCL's footprint), reserve_cus 0 / 8 / 16
set -o pipefail
out=gpurun_out/${1:-cumask}
shift
mkdir -p $out
steps=${@:-probe split}
for st in $steps; do
  case $st in
    probe) timeout -k 10 300 python -u bench/cumask_probe.py > $out/probe.jsonl 2> $out/probe.err || exit 1 ;;
    split)
      for g in 16384 4096; do
        timeout -k 10 300 python -u bench/pipe_latency.py --grid $g --world 8 --rank 3 --recurrences 1 --graphs 1 \
          --overlaps 1 --fat 1 --delays 10 --halo-us 30 --iters 640 --reserve-cus 0,32 --halo-ahead 0,1 \
          >> $out/split.jsonl 2>> $out/split.err || exit 1
        timeout -k 10 300 python -u bench/pipe_latency.py --grid $g --world 8 --rank 3 --recurrences 1 --graphs 1 \
          --overlaps 0 --fat 1 --delays 10 --halo-us 30 --iters 640 --reserve-cus 0 \
          >> $out/split.jsonl 2>> $out/split.err || exit 1
      done
      timeout -k 10 300 python -u bench/pipe_latency.py --problem poisson3d --grid 512 --world 8 --rank 3 --recurrences 1 \
        --graphs 1 --overlaps 1 --fat 1 --delays 10 --halo-us 30 --iters 640 --reserve-cus 0,32 --halo-ahead 0,1 \
        >> $out/split.jsonl 2>> $out/split.err || exit 1 ;;
    full)
      for rc in 0 32 64; do
        timeout -k 10 300 python -u bench.py --steps 64 --warmup 8 --set reserve_cus=$rc > $out/bench_rc$rc.json 2>> $out/bench.err || exit 1
      done
      for rc in 0 32; do
        timeout -k 10 300 python -u bench.py --grid 4096 --steps 640 --warmup 64 --set reserve_cus=$rc > $out/bench4096_rc$rc.json 2>> $out/bench.err || exit 1
        timeout -k 10 300 python -u bench.py --problem poisson3d --grid 512 --steps 64 --warmup 8 --set reserve_cus=$rc > $out/bench512_rc$rc.json 2>> $out/bench.err || exit 1
      done ;;
    pipe)
      timeout -k 10 300 python -u bench/pipe_latency.py --problem randspd --recurrences 1,2 --graphs 1 --fat 1 \
        --delays 20,40 --reserve-cus 0,32 --iters 640 >> $out/pipe.jsonl 2>> $out/pipe.err || exit 1
      timeout -k 10 300 python -u bench/pipe_latency.py --grid 4096 --recurrences 1,2 --graphs 1 --fat 1 \
        --delays 20,40 --reserve-cus 0,32 --iters 640 >> $out/pipe.jsonl 2>> $out/pipe.err || exit 1 ;;
    corun)
      for rc in 0 32; do
        timeout -k 10 300 python -u bench/corun_probe.py --set reserve_cus=$rc > $out/corun_rc$rc.json 2>> $out/corun.err || exit 1
      done ;;
  esac
done
