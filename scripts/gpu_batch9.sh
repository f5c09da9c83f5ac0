#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step tests 900 python -m pytest tests/test_gpu_kernels.py -x -q
step smoke 600 python -c "import __graft_entry__ as g; g.smoke()"
step b4096 600 python bench.py --grid 4096 --steps 2000 --warmup 100
step b4096_classic 600 python bench.py --grid 4096 --steps 2000 --warmup 100 --recurrence 0
step b8192 600 python bench.py --grid 8192 --steps 500 --warmup 50
