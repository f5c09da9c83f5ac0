#!/usr/bin/env python3
"""Where the config-5 tile SpMV's time goes: y = A x through the tiles (k_tiles MODE 1, the
true-residual SpMV) on a P = 8 rank's share of the scrambled random SPD, timed over --reps calls of
true_residual_norm() (one tile sweep + a norm each).  With MCG_TILES_ABLATE set the sweep drops parts
of its work (cg_tiles.hip ABL bits: 1 LDS adds, 2 gathers, 4 pacing, 8 tile loads; results wrong),
so the differences say what each part costs.  One JSON line.
    MCG_TILES_ABLATE=3 python bench/tiles_ablate.py
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--band", type=int, default=410)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    import torch

    import cuda_mpi_parallel_amd as mcg

    torch.cuda.init()
    C = mcg.native()
    spec = mcg.make_problem("randspd", rows=a.rows, band=a.band, density=1.0, scramble=1, rhs="random")
    o = C.CgOptions(maxit=1 << 30, tol=-1.0, check_every=1 << 30, format="sellc8", recurrence=-1)
    for kv in a.set:
        k, v = kv.split("=", 1)
        setattr(o, k, type(getattr(o, k))(v))
    s = C.Solver(spec.native(), o, 3, 8, C.NullComm(3, 8))
    s.setup()
    s.reset()
    s.true_residual_norm()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        v = s.true_residual_norm()
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / a.reps
    info = s.info
    print(json.dumps({"ablate": int(os.environ.get("MCG_TILES_ABLATE", "0")), "ms_per_spmv": round(ms, 3),
                      "tiles": info.get("tiles"), "nnz_local": info.get("nnz_local"), "value": v}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
