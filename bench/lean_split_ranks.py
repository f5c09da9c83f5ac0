"""lean_split at P LocalComm ranks (forced, lean_split = 1) against the generic pass: relative rnorm
gap after a fixed iteration count, with and without the halo overlap.  One JSON line per arm.
    python bench/lean_split_ranks.py [--n 2048] [--world 4] [--iters 40]
"""
import argparse
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cuda_mpi_parallel_amd as mcg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=2048)
ap.add_argument("--world", type=int, default=4)
ap.add_argument("--iters", type=int, default=40)
ap.add_argument("--lines", default="100,1500", help="grid lines holding a changed diagonal entry")
a = ap.parse_args()
n = a.n
T = sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(n, n))
I = sp.identity(n)
A = (sp.kron(I, T) + sp.kron(T, I)).tolil()
d = A.diagonal()
for ln in [int(x) for x in a.lines.split(",")]:
    d[n * ln + 7] += 0.5
A.setdiag(d)
p = mcg.csr_problem(A.tocsr(), b=np.ones(n * n))
C = mcg.native()
base = None
for w, ls in ((1, 0), (1, 1), (2, 0), (2, 1)):
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1)
    o.lean_split = ls
    out = C.run_local_ranks(p.native(), o, w, a.iters, True)
    print(json.dumps({"arm": f"P{w}_ls{ls}", "rnorm": out["ranks"][0]["rnorm"],
                      "split": [rk["lean_split"] for rk in out["ranks"]]}), flush=True)
for tag, ls, ov in (("generic", 0, True), ("split", 1, True), ("split_noov", 1, False), ("generic_noov", 0, False)):
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1)
    o.lean_split = ls
    o.overlap = ov
    out = C.run_local_ranks(p.native(), o, a.world, a.iters, True)
    r = out["ranks"][0]["rnorm"]
    if base is None:
        base = r
    print(json.dumps({"arm": tag, "rnorm": r, "gap": abs(r - base) / base,
                      "split": [rk["lean_split"] for rk in out["ranks"]],
                      "lean_only": [rk["lean_only"] for rk in out["ranks"]]}), flush=True)
