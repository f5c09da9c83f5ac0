#!/bin/bash
source scripts/gpu_check.sh
export TMPDIR=/tmp
step pytest_mr 900 python -m pytest tests/test_gpu_multirank.py -x -q
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
