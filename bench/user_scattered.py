"""A scattered user CSR (the reference's input form, CUDACG.cu:93-117) at P = 1: the scrambled random
SPD family exported to a host CSR and handed to the solver as a user matrix, timed with the
L2-segment tiles (auto for scattered user matrices) against the plain SELL-64 split pass and CSR.

    python bench/user_scattered.py --rows 4000000 --band 64 --density 0.5 --iters 100
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--band", type=int, default=64)
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401

    import cuda_mpi_parallel_amd as mcg

    C = mcg.native()
    spec = mcg.make_problem("randspd", rows=a.rows, band=a.band, density=a.density, scramble=1, rhs="random")
    t0 = time.perf_counter()
    rp, cols, vals = C.host_csr(spec.native())
    b = C.host_rhs(spec.native(), 0, a.rows)
    H = C.HostMatrix(np.asarray(rp, np.int64), np.asarray(cols, np.int64), np.asarray(vals, np.float64), b)
    build_s = time.perf_counter() - t0
    prob = mcg.models.CsrProblem(H, "reference", 1234)
    nnz = int(rp[-1])
    print(json.dumps({"rows": a.rows, "nnz": nnz, "far_entries": H.far_entries, "bandwidth": H.bandwidth,
                      "host_build_s": round(build_s, 1)}), flush=True)
    for name, kw in (("tiles (auto)", dict(format="sell", recurrence=1)),
                     ("SELL-64 split", dict(format="sell", recurrence=1, tiles=0)),
                     ("CSR split", dict(format="csr", recurrence=1, tiles=0))):
        s = mcg.CGSolver(prob, tol=-1.0, maxit=1 << 30, **kw)
        s.reset()
        s.run(10)
        s.synchronize()
        t = time.perf_counter()
        s.run(a.iters)
        s.synchronize()
        dt = time.perf_counter() - t
        s.finalize()
        res = s.result()
        tr = s.true_residual_norm()
        print(json.dumps({"form": name, "tiles": s.info["tiles"], "format": s.info["format"], "pmat": s.info["pmat"],
                          "it_per_s": round(a.iters / dt, 2), "ms_per_iter": round(1e3 * dt / a.iters, 3),
                          "rnorm": res["rnorm"], "true_rnorm": tr}), flush=True)
        del s


if __name__ == "__main__":
    main()
