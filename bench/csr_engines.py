#!/usr/bin/env python3
"""CSR engines on a user matrix with skewed row lengths (GPU): iterations/s of the single- and
two-reduction CSR passes with the thread-per-row (1), CSR-vector (2) and row-length-adaptive (4)
engines.  The matrix: a random SPD pattern of short rows (~`deg` entries) plus `hubs` rows coupled
to `hub_deg` columns each (power-law-like skew), built with SciPy on the host.

  python bench/csr_engines.py --rows 2000000 --hubs 2000 --hub-deg 2000
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp


def skewed(n: int, deg: int, hubs: int, hub_deg: int, seed: int = 11) -> sp.csr_matrix:
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(n), deg)
    cols = rng.integers(0, n, size=n * deg)
    h = rng.choice(n, hubs, replace=False)
    hr = np.repeat(h, hub_deg)
    hc = rng.integers(0, n, size=hubs * hub_deg)
    r = np.concatenate([rows, hr])
    c = np.concatenate([cols, hc])
    keep = r != c
    r, c = r[keep], c[keep]
    v = -rng.random(r.size) * 1e-3
    A = sp.coo_matrix((v, (r, c)), shape=(n, n)).tocsr()
    A = A + A.T
    A.sum_duplicates()
    d = np.asarray(abs(A).sum(axis=1)).ravel() + 1.0
    return (A + sp.diags(d)).tocsr()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--deg", type=int, default=4)
    ap.add_argument("--hubs", type=int, default=2000)
    ap.add_argument("--hub-deg", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import cuda_mpi_parallel_amd as mcg

    A = skewed(a.rows, a.deg, a.hubs, a.hub_deg)
    lens = np.diff(A.indptr)
    p = mcg.csr_problem(A, rhs="random")
    out = {"rows": a.rows, "nnz": int(A.nnz), "max_row": int(lens.max()), "mean_row": round(float(lens.mean()), 2)}
    for rec in (1, 0):
        for v in (1, 2, 4):
            s = mcg.CGSolver(p, format="csr", recurrence=rec, tol=-1.0, maxit=1 << 30, spmv_variant=v,
                             check_every=1 << 30)
            s.reset()
            s.run(10)
            s.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.run(a.iters)
            s.synchronize()
            dt = time.perf_counter() - t0
            out[f"rec{rec}_v{v}"] = round(a.iters / dt, 2)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
