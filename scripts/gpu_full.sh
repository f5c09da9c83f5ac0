#!/bin/bash
# full GPU suite + headline bench + ~200 GB random-SPD run (BASELINE.json config 5 per-GPU size)
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 1100 python -m pytest tests -m gpu -x -q
step bench 600 python bench.py
step bench3d 600 python bench.py --problem poisson3d --grid 512
step rs200 900 python bench.py --problem randspd --rows 12500000 --band 4096 --density 0.2 --steps 20 --warmup 3
