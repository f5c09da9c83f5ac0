#!/usr/bin/env python3
"""Rehearse the distributed path at the headline size on ONE GPU: P ranks as threads sharing the
device (LocalComm: D2D halo copies + fixed-order all-reduce), fixed iterations, then every rank's
true residual ||b - A x|| against the recurrence residual and the P = 1 run.  Correctness only
(the ranks share one GPU, so no timing is reported).

  python bench/rehearse_ranks.py --n 16384 --iters 40 --world 1 2 8
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cuda_mpi_parallel_amd as mcg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--problem", default="poisson2d")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--world", type=int, nargs="+", default=[1, 2, 8])
    ap.add_argument("--grid", type=int, default=None, help="alias of --n")
    ap.add_argument("--rows", type=int, default=2_000_000, help="randspd rows")
    ap.add_argument("--band", type=int, default=100, help="randspd candidate offsets per side")
    ap.add_argument("--density", type=float, default=1.0)
    ap.add_argument("--spread", type=int, default=-1, help="randspd spread (-1 = rows: unstructured)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="collectives in one stream order (what --comm single runs at P > 1)")
    ap.add_argument("--phases", type=int, default=0,
                    help="> 0: per-rank phase timing (interior || halo, boundary wait) over that many iterations")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    C = mcg.native()
    if args.problem == "randspd":
        spec = mcg.make_problem("randspd", rows=args.rows, band=args.band, density=args.density,
                                spread=args.rows if args.spread < 0 else args.spread)
    else:
        spec = mcg.make_problem(args.problem, n=args.grid or args.n)
    ref = None
    for w in args.world:
        o = C.CgOptions(maxit=1 << 30, tol=-1.0, format="sellc8", recurrence=1, check_every=1 << 30,
                        overlap=not args.no_overlap)
        out = C.run_local_ranks(spec.native(), o, w, args.iters, True, args.phases)
        r = out["ranks"]
        rn = r[0]["rnorm"]
        tr = max(x["true_rnorm"] for x in r)
        ok = all(x["iterations"] == args.iters + args.phases for x in r) and abs(tr - rn) <= 1e-6 * max(tr, 1e-300)
        if ref is None:
            ref = rn
        line = {"world": w, "overlap": not args.no_overlap, "iterations": r[0]["iterations"], "rnorm": rn, "true_rnorm": tr,
                "rel_vs_first": abs(rn - ref) / ref, "ok": ok,
                "lean_only": all(x.get("lean_only", False) for x in r)}
        if args.phases:  # worst rank per phase (the ranks share one GPU: relative sizes, not speed)
            keys = sorted(r[0]["phases"])
            line["phase_us_max"] = {k: round(max(x["phases"][k] for x in r), 2) for k in keys}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
