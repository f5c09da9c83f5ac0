#!/bin/bash
source scripts/gpu_check.sh
step cli_demo 120 ./bin/mcg-cg
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step bench_n4096 300 python bench.py --n 4096 --steps 200 --warmup 20
step bench_csr 600 python bench.py --steps 100 --warmup 10
step bench_sell 600 python bench.py --steps 100 --warmup 10 --format sell
