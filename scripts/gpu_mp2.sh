#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step mp2 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --grid 2048 --steps 20 --warmup 4 --format sell16
