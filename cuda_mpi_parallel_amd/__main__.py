"""``python -m cuda_mpi_parallel_amd`` — the reference's entry point, process-per-GPU flavour.

With no arguments it behaves like the reference binary (CUDACG.cu:41-366): solve the
built-in 3x3 system on GPU 0, print x one ``%f`` per line, then ``Success``.  Under
``torchrun --nproc-per-node N`` every process drives one GPU and the ranks talk over
RCCL (the native ``bin/mcg-cg --gpus N`` runs the same solver with one thread per GPU).
Failures print one line to stdout and exit 1, like the reference's CLEANUP path.
"""
from __future__ import annotations

import argparse
import json
import sys


def _parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m cuda_mpi_parallel_amd", allow_abbrev=False)
    ap.add_argument("--problem", default="demo", choices=["demo", "poisson2d", "poisson3d", "randspd"])
    ap.add_argument("--grid", "--N", dest="grid", type=int, default=None, help="grid edge N")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--band", type=int, default=None)
    ap.add_argument("--density", type=float, default=None)
    ap.add_argument("--rhs", default=None, choices=["reference", "random", "ones"])
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--sim-ranks", type=int, default=1, help="CPU path: virtual ranks")
    ap.add_argument("--maxit", type=int, default=2000)
    ap.add_argument("--tol", type=float, default=1e-7)
    ap.add_argument("--check-every", type=int, default=32)
    ap.add_argument("--format", default=None, choices=["csr", "sell", "sell16", "sellc8"],
                    help="default: csr for the demo (reference layout), sellc8 for generated problems")
    ap.add_argument("--rtol", type=float, default=0.0, help="> 0: stop on ||r|| < rtol * ||b||")
    ap.add_argument("--recurrence", type=int, default=-1)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--checkpoint", default="")
    ap.add_argument("--checkpoint-every", type=int, default=0)
    ap.add_argument("--resume", default="")
    ap.add_argument("--print-x", default="auto", choices=["auto", "yes", "no"])
    ap.add_argument("--report", default="text", choices=["text", "json"])
    ap.add_argument("--verify", action="store_true")
    return ap


def main(argv=None) -> int:
    args = _parser().parse_args(argv)
    try:
        import numpy as np

        import cuda_mpi_parallel_amd as mcg
        from cuda_mpi_parallel_amd.parallel import dist as pdist

        kw = {k: v for k, v in dict(n=args.grid, rows=args.rows, band=args.band, density=args.density,
                                     rhs=args.rhs).items() if v is not None}
        spec = mcg.make_problem(args.problem, seed=args.seed, **kw)
        n = spec.n_rows
        want_x = args.print_x == "yes" or (args.print_x == "auto" and n <= 1000)
        env = pdist.dist_env()
        true_rnorm = None
        if args.device == "cpu":
            C = mcg.native()
            o = C.CgOptions(maxit=args.maxit, tol=args.tol)
            o.rtol = args.rtol
            res = (C.cpu_cg_partitioned(spec.native(), args.sim_ranks, o) if args.sim_ranks > 1
                   else C.cpu_cg(spec.native(), o))
            x = res["x"]
            rank = 0
        else:
            s = mcg.CGSolver(spec, maxit=args.maxit, tol=args.tol, check_every=args.check_every,
                             overlap=not args.no_overlap, use_graph=not args.no_graph,
                             format=args.format or ("csr" if args.problem == "demo" else "sellc8"),
                             recurrence=args.recurrence, rtol=args.rtol, checkpoint_every=args.checkpoint_every,
                             checkpoint_path=args.checkpoint)
            if args.resume:
                s.load_checkpoint(args.resume)
            res = s.solve(resume=bool(args.resume))
            if args.verify:
                true_rnorm = s.true_residual_norm()
            x = res["x_local"]
            rank = env.rank
            if env.world > 1 and want_x:
                from cuda_mpi_parallel_amd.parallel.cpu_ref import gather_x

                x = gather_x({"row_begin": res["row_begin"], "x": x})
        if rank == 0:
            out = []
            if want_x:
                out.append("".join("%f\n" % v for v in np.asarray(x)))
            if args.report == "json":
                out.append(json.dumps({"problem": spec.problem, "n": n, "ranks": env.world if args.device == "gpu"
                                       else args.sim_ranks, "device": args.device, "iterations": res["iterations"],
                                       "converged": res["converged"], "breakdown": res["breakdown"],
                                       "rnorm": res["rnorm"], "true_rnorm": true_rnorm,
                                       "solve_s": res["solve_seconds"], "it_per_s": res["iters_per_second"]}) + "\n")
            out.append("Success\n")  # CUDACG.cu:365
            sys.stdout.write("".join(out))
            sys.stdout.flush()
        return 0
    except Exception as e:  # one line on stdout, exit 1 (CUDACG.cu:10-33 CLEANUP semantics)
        msg = str(e).split(" [")[0]
        print(msg if msg else type(e).__name__)
        return 1


if __name__ == "__main__":
    sys.exit(main())
