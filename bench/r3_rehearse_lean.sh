#!/bin/bash
# r3: the distributed path with the lean kernels at the headline sizes, P = 1/2/4/8 ranks on one GPU
# (LocalComm), fixed iterations, in the default one-stream order: residuals vs P = 1, true residual
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3reh}
mkdir -p $O
timeout -k 10 400 python bench/rehearse_ranks.py --n 16384 --iters 40 --world 1 2 4 8 --no-overlap > $O/rehearse_16384.jsonl 2> $O/err_16384.txt || exit 1
timeout -k 10 400 python bench/rehearse_ranks.py --problem poisson3d --n 512 --iters 40 --world 1 2 4 8 --no-overlap > $O/rehearse_512.jsonl 2> $O/err_512.txt || exit 1
echo done
