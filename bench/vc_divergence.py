#!/usr/bin/env python3
"""How far do CG residual histories of the variable-coefficient 2-D operator drift apart from rounding
alone?  The same problem (poisson2d --coef 1, 1024^2, random RHS) through four solvers:

  cpu    the CPU oracle, op for op the reference's two-reduction CG (CUDACG.cu:269-352)
  csr0   the GPU two-reduction pass on CSR (the reference's algorithm; only the dot products' block
         order differs from the oracle)
  d16    the GPU single-reduction pass on SELL-64/d16 (generic kernels)
  diav   the GPU default: SELL-64/diav three-term Ap-recomputing line carry (lean runs)

and prints |rnorm_k - cpu_k| / cpu_k at several k, plus each run's recurrence vs ||b - A x||, and (r5,
VERDICT r4 item 9) each GPU run against the GPU csr0 run -- the same rounding growth, both on the GPU:
|rnorm_k - csr0_k| / csr0_k and ||x_k - x_csr0,k|| / ||x_csr0,k||.  One JSON line.  A pure-rounding drift
shows as csr0 drifting like the others.
    python bench/vc_divergence.py [--n 1024]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--coef", type=int, default=1)
    ap.add_argument("--its", default="20,50,100,200,300,500,1000,2000")
    a = ap.parse_args()
    import numpy as np

    import cuda_mpi_parallel_amd as mcg

    its = [int(x) for x in a.its.split(",")]
    spec = mcg.make_problem("poisson2d", n=a.n, coef=a.coef, rhs="random")
    C = mcg.native()
    cpu = C.cpu_cg(spec.native(), C.CgOptions(maxit=max(its), tol=-1.0))
    hist = np.asarray(cpu["rnorm_history"])
    arms = {"csr0": dict(format="csr", recurrence=0), "d16": dict(format="sellc8", recurrence=1, carry_vc=0),
            "diav": dict(format="sellc8", recurrence=1)}
    out = {"n": a.n, "coef": a.coef, "cpu_rnorm": {k: float(hist[k - 1]) for k in its}, "gap": {}, "true_gap": {}}
    ref = {}  # csr0's (rnorm, x) per k
    for name, kw in arms.items():
        s = mcg.CGSolver(spec, tol=-1.0, maxit=max(its), **kw)
        gaps = {}
        for k in its:
            s.reset()
            s.run(k)
            s.finalize()
            r = s.result()["rnorm"]
            gaps[k] = abs(r - hist[k - 1]) / hist[k - 1]
            x = np.asarray(s._s.x_local())
            if name == "csr0":
                ref[k] = (r, x)
            else:
                r0, x0 = ref[k]
                out.setdefault("gap_vs_csr0", {}).setdefault(name, {})[k] = abs(r - r0) / r0
                out.setdefault("xgap_vs_csr0", {}).setdefault(name, {})[k] = float(np.linalg.norm(x - x0) / np.linalg.norm(x0))
        tr = s.true_residual_norm()
        out["gap"][name] = gaps
        out["true_gap"][name] = abs(tr - s.result()["rnorm"]) / tr
        out.setdefault("info", {})[name] = {k: s.info.get(k) for k in ("format", "diav", "lean_only", "recurrence")}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
