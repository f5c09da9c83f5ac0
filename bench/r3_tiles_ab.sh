#!/bin/bash
# scrambled config-5 share (rank 3 of 8), tile SpMV A/B on one box: two repeats + the tiles GPU tests
set -o pipefail
out=gpurun_out/${1:-tab}
mkdir -p $out
S="--problem randspd --rows 100000000 --band 410 --density 1.0 --scramble 1 --sim-world 8 --sim-rank 3 --steps 6 --warmup 2 --phases 0"
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py $S > $out/c5_$rep.json 2>> $out/err.log || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_irregular.py -x -q --timeout 300 --timeout-method thread > $out/pytest_irregular.txt 2>&1 || exit 1
