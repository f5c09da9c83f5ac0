#!/usr/bin/env python3
"""A/B of the lean / generic split on a user matrix that is a 2-D Laplacian except for a few rows.

One changed diagonal entry leaves one slice of one run off the uniform pattern: without the split the
whole pass drops to the generic three-term kernels (the round-3 cliff, profiles/r3/lean: 581 vs 515
it/s at 16384^2); with it (lean_split, the default) only that run does.  Arms, same matrix and RHS:

  uniform   the unperturbed Laplacian (every run lean; the ceiling)
  generic   the perturbed matrix, lean_split = 0 (the pre-split dispatch)
  side      the perturbed matrix, lean_split = 1, the generic launch on a side stream beside it (r6: three
            p buffers when the split allows them, the default)
  two       the same with two p buffers (p3buf = 0: the r5 split)
  sideplain the split's r4 geometry (one grid by the runs' length, no packed edges: two p buffers since late r6)
  rsv8/32   side with 8 / 32 CUs withheld from the lean launch's stream (the generic launch's side stream
            keeps them: its pieces start at once instead of after the lean launch's workgroups)
  serial    side with the generic launch ahead of the lean one on one stream
  stream    side with the generic launch beside the lean one on the side stream (r6's first form; the
            default since is one combined launch, the generic ranges' workgroups first)

Prints one JSON line with it/s per arm (fixed iteration count, untimed warmup).
    python bench/lean_split_ab.py [--n 8192] [--spots 3] [--steps 400] [--sim-world 8 --sim-rank 3]
--sim-world P --sim-rank r: rank r's share of a P-rank job alone on the GPU (collectives that move nothing,
the in-kernel halo on, as bench.py --sim-world ... --set halo_pull=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _laplacian(n):
    import scipy.sparse as sp
    T = sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(n, n), format="csr")
    I = sp.identity(n, format="csr")
    return (sp.kron(I, T, format="csr") + sp.kron(T, I, format="csr")).tocsr()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--spots", type=int, default=3)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--arms", default="uniform,generic,side,two", help="comma list of arms to run")
    ap.add_argument("--sim-world", type=int, default=0)
    ap.add_argument("--sim-rank", type=int, default=0)
    a = ap.parse_args()
    import numpy as np

    import cuda_mpi_parallel_amd as mcg

    t0 = time.perf_counter()
    A = _laplacian(a.n)
    print(json.dumps({"built": a.n, "nnz": int(A.nnz), "s": round(time.perf_counter() - t0, 1)}), flush=True)
    rng = np.random.default_rng(7)
    spots = rng.integers(0, a.n * a.n, a.spots)
    out = {"n": a.n, "spots": a.spots, "steps": a.steps, "its": {}, "info": {}, "sim": [a.sim_rank, a.sim_world]}
    arms = [("uniform", {})] + [(f"generic_{i}", {"lean_split": 0}) for i in range(a.reps)]
    arms += [(f"side_{i}", {"lean_split": 1}) for i in range(a.reps)]
    arms += [(f"two_{i}", {"lean_split": 1, "p3buf": 0}) for i in range(a.reps)]
    arms += [(f"sideplain_{i}", {"lean_split": 1, "lean_packed": 0}) for i in range(a.reps)]
    arms += [(f"rsv{c}_{i}", {"lean_split": 1, "reserve_cus": c}) for i in range(a.reps) for c in (8, 32)]
    arms += [(f"serial_{i}", {"lean_split": 1, "split_serial": 1}) for i in range(a.reps)]
    arms += [(f"stream_{i}", {"lean_split": 1, "split_serial": 0}) for i in range(a.reps)]
    want = set(a.arms.split(","))
    arms = [(nm, kw) for nm, kw in arms if nm.split("_")[0] in want]
    for name, kw in arms:
        if name != "uniform" and spots is not None:
            # one matrix in memory (16384^2: 1.3 G nnz): the changed diagonal entries, in place
            for r in spots:
                lo, hi = A.indptr[r], A.indptr[r + 1]
                A.data[lo + int(np.nonzero(A.indices[lo:hi] == r)[0][0])] += 0.5
            spots = None
        p = mcg.csr_problem(A, rhs="random")
        if a.sim_world > 1:
            from cuda_mpi_parallel_amd.solver import _opts

            C = mcg.native()
            o = _opts(maxit=a.steps + a.warmup, tol=-1.0, format="sellc8", recurrence=1, halo_pull=1, **kw)
            s = mcg.CGSolver.__new__(mcg.CGSolver)  # the rank's share on a NullComm, as bench.py --sim-world
            s._s = C.Solver(p.native(), o, a.sim_rank, a.sim_world, C.NullComm(a.sim_rank, a.sim_world))
            s._s.setup()
        else:
            s = mcg.CGSolver(p, format="sellc8", recurrence=1, tol=-1.0, maxit=a.steps + a.warmup, **kw)
        s.reset()
        s.run(a.warmup)
        s.synchronize()
        t0 = time.perf_counter()
        s.run(a.steps)
        s.synchronize()
        dt = time.perf_counter() - t0
        out["its"][name] = round(a.steps / dt, 1)
        out["info"][name] = {k: s.info.get(k) for k in ("lean_only", "lean_split", "dia_uniform", "lean_mix", "p3buf")}
        del s, p
        print(json.dumps({"arm": name, "it_s": out["its"][name]}), flush=True)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
