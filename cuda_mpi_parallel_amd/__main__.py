"""``python -m cuda_mpi_parallel_amd`` — the reference's entry point, process-per-GPU flavour.

With no arguments it behaves like the reference binary (CUDACG.cu:41-366): solve the
built-in 3x3 system on GPU 0, print x one ``%f`` per line, then ``Success``.  ``--gpus P``
starts P ranks (one process per GPU, parallel/launch.py; or run it under ``torchrun``) that
talk over RCCL; the native ``bin/mcg-cg --gpus P`` runs the same solver with one thread per
GPU.  Both CLIs take the flag table of ``cli_spec.py``.  Failures print one line to stdout and
exit 1, like the reference's CLEANUP path (CUDACG.cu:10-33).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

from .cli_spec import FLAGS, recurrence, tri
from .utils import format_x

SWITCHES = {"--no-overlap", "--no-graph", "--force-comm", "--verify", "--rehearse-ranks"}
CHOICES = {"--problem": ["demo", "poisson2d", "poisson3d", "randspd", "csr", "random-spd", "random"],
           "--rhs": ["reference", "random", "ones"], "--device": ["gpu", "cpu"],
           "--format": ["csr", "sell", "sell16", "sellc8"], "--print-x": ["auto", "yes", "no"],
           "--report": ["text", "json"], "--comm": ["dual", "single"], "--halo-mode": ["auto", "window", "allgather", "-1", "0", "1"],
           "--halo-transport": ["auto", "rccl"], "--allreduce": ["auto", "rccl", "ipc"],
           "--transport-probe": ["auto", "off", "on", "-1", "0", "1"]}
INTS = {"--n", "--rows", "--band", "--spread", "--scramble", "--coef", "--seed", "--gpus", "--sim-ranks", "--maxit", "--check-every",
        "--fixed-iters", "--warmup", "--blocks-per-cu", "--spmv-variant", "--checkpoint-every", "--inject-nan-at",
        "--pipe-rr", "--reserve-cus"}
FLOATS = {"--density", "--nnz-per-row", "--tol", "--rtol", "--watchdog"}
DEFAULTS = {"--problem": "demo", "--seed": 1234, "--device": "gpu", "--gpus": None, "--sim-ranks": 1,
            "--maxit": 2000, "--tol": 1e-7, "--rtol": 0.0, "--check-every": 32, "--fixed-iters": 0, "--warmup": 0,
            "--watchdog": 0.0, "--recurrence": "auto", "--interleave": "auto", "--window": "auto", "--carry": "auto",
            "--pmat": "auto", "--fused-reduce": "auto", "--halo-mode": "auto", "--blocks-per-cu": 0,
            "--spmv-variant": -1, "--checkpoint": "", "--checkpoint-every": 0, "--resume": "", "--inject-nan-at": -1,
            "--print-x": "auto", "--report": "text", "--comm": "single", "--pipe-rr": 0,
            "--reserve-cus": 0, "--halo-transport": "auto", "--allreduce": "auto", "--transport-probe": "auto"}


def _parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m cuda_mpi_parallel_amd", allow_abbrev=False)
    for flag, _example, help_ in FLAGS:
        names = [flag] + (["--grid", "--N"] if flag == "--n" else [])
        if flag in SWITCHES:
            ap.add_argument(*names, action="store_true", help=help_)
            continue
        kw = dict(help=help_, default=DEFAULTS.get(flag))
        if flag in INTS:
            kw["type"] = int
        elif flag in FLOATS:
            kw["type"] = float
        if flag in CHOICES:
            kw["choices"] = CHOICES[flag]
        ap.add_argument(*names, **kw)
    return ap


def _spec(args):
    import cuda_mpi_parallel_amd as mcg

    if args.matrix or args.problem == "csr":
        if not args.matrix:
            raise ValueError("invalid arguments: --problem csr needs --matrix FILE")
        H = mcg.native().HostMatrix.read_mtx(args.matrix)
        if args.rhs_file:
            H = _with_rhs(mcg, H, mcg.native().read_vector(args.rhs_file))
        return mcg.models.CsrProblem(H, args.rhs or "reference", args.seed)
    kw = {"seed": args.seed}
    if args.rhs:
        kw["rhs"] = args.rhs
    problem = {"random-spd": "randspd", "random": "randspd"}.get(args.problem, args.problem)
    if problem in ("poisson2d", "poisson3d") and args.n is not None:
        kw["n"] = args.n
    if problem in ("poisson2d", "poisson3d") and args.coef:
        kw["coef"] = args.coef
    if problem == "randspd":
        for k in ("rows", "band", "density", "spread", "scramble"):
            v = getattr(args, k)
            if v is not None:
                kw[k] = v
        if args.nnz_per_row is not None:
            kw["nnz_per_row"] = args.nnz_per_row
    return mcg.make_problem(problem, **kw)


def _with_rhs(mcg, H, b):
    """A HostMatrix with the same CSR and right-hand side b (the native class is immutable here)."""
    import numpy as np

    from .models import CsrProblem, host_csr

    rowptr, cols, vals = host_csr(CsrProblem(H))
    return mcg.native().HostMatrix(rowptr, cols.astype(np.int64), vals, b)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    args = _parser().parse_args(argv)
    if args.device == "gpu":
        from .parallel import launch

        rc = launch.launch_or_none(args.gpus, argv, module="cuda_mpi_parallel_amd", share_device=args.rehearse_ranks)
        if rc is not None:
            return rc
    try:
        return _run(args)
    except Exception as e:  # one line on stdout, exit 1 (CUDACG.cu:10-33 CLEANUP semantics)
        msg = str(e).split(" [")[0]
        print(msg if msg else type(e).__name__)
        return 1


def _run(args) -> int:
    import numpy as np

    import cuda_mpi_parallel_amd as mcg
    from cuda_mpi_parallel_amd.parallel import dist as pdist

    spec = _spec(args)
    n = spec.n_rows
    want_x = args.print_x == "yes" or (args.print_x == "auto" and n <= 1000)
    env = pdist.dist_env()
    true_rnorm = None
    info = {}
    C = mcg.native()
    fixed = args.fixed_iters > 0
    maxit, tol = (args.fixed_iters, -1.0) if fixed else (args.maxit, args.tol)
    if args.device == "cpu":
        o = C.CgOptions(maxit=maxit, tol=tol)
        o.rtol = args.rtol
        o.halo_mode = _halo(args.halo_mode)
        res = (C.cpu_cg_partitioned(spec.native(), args.sim_ranks, o) if args.sim_ranks > 1
               else C.cpu_cg(spec.native(), o))
        x = res["x"]
        rank, world = 0, args.sim_ranks
    else:
        s = mcg.CGSolver(spec, maxit=maxit, tol=tol, check_every=args.check_every, overlap=not args.no_overlap,
                         use_graph=not args.no_graph, force_comm=args.force_comm, comm_mode=args.comm,
                         format=args.format or ("csr" if spec.problem == "demo" else "sellc8"),
                         blocks_per_cu=args.blocks_per_cu, spmv_variant=args.spmv_variant,
                         recurrence=recurrence(args.recurrence) if spec.problem != "demo" or args.recurrence != "auto"
                         else 0,
                         interleave=tri(args.interleave), window=tri(args.window), carry=tri(args.carry),
                         pmat=tri(args.pmat), fused_reduce=tri(args.fused_reduce), halo_mode=_halo(args.halo_mode),
                         rtol=args.rtol, pipe_rr=args.pipe_rr, checkpoint_every=args.checkpoint_every, checkpoint_path=args.checkpoint,
                         inject_nan_at=args.inject_nan_at, watchdog_seconds=args.watchdog,
                         reserve_cus=args.reserve_cus, halo_transport=args.halo_transport, allreduce=args.allreduce,
                         rehearse_ranks=args.rehearse_ranks,
                         transport_probe=0 if tri(args.transport_probe) == 0 else -1)
        if fixed:
            import torch.distributed as dist

            s.reset()
            s.run(args.warmup)
            s.synchronize()
            if env.world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            s.run(args.fixed_iters)
            s.synchronize()
            if env.world > 1:
                dist.barrier()
            dt = time.perf_counter() - t0
            s.finalize()
            res = s.result()
            res["solve_seconds"] = dt
            res["iters_per_second"] = args.fixed_iters / dt if dt > 0 else 0.0
            res["x_local"] = s.x_local()
            res["row_begin"] = s.layout["row_begin"]
        else:
            if args.resume:
                s.load_checkpoint(args.resume)
            res = s.solve(resume=bool(args.resume))
        if args.verify:
            true_rnorm = s.true_residual_norm()
        info = s.info
        x = res["x_local"]
        rank, world = env.rank, env.world
        if env.world > 1 and want_x:
            from cuda_mpi_parallel_amd.parallel.cpu_ref import gather_x

            x = gather_x({"row_begin": res["row_begin"], "x": x})
    if rank == 0:
        out = []
        if want_x:
            out.append(format_x(np.asarray(x)))
        if args.report == "json":
            out.append(json.dumps({
                "problem": spec.problem, "n": n, "nnz_rank0": info.get("nnz_local", 0), "ranks": world,
                "device": args.device, "format": "csr" if args.device == "cpu" else info.get("format"),
                "iterations": res["iterations"], "converged": res["converged"], "breakdown": res["breakdown"],
                "rnorm": res["rnorm"], "true_rnorm": true_rnorm, "setup_s": res.get("setup_seconds"),
                "solve_s": res["solve_seconds"], "it_per_s": res["iters_per_second"],
                "device_bytes_rank0": info.get("device_bytes", 0), **_transport_report(info, world, args)}) + "\n")
        elif not want_x or n > 3:
            sys.stderr.write("[mcg] problem=%s n=%d ranks=%d iterations=%d converged=%d rnorm=%.3e solve=%.4fs "
                             "(%.2f it/s)\n" % (spec.problem, n, world, res["iterations"], int(res["converged"]),
                                                res["rnorm"], res["solve_seconds"], res["iters_per_second"]))
        out.append("Success\n")  # CUDACG.cu:365
        sys.stdout.write("".join(out))
        sys.stdout.flush()
    return 0


def _transport_report(info, world, args) -> dict:
    """The P > 1 transports in effect (the keys bin/mcg-cg --report json prints too)."""
    gpu = args.device == "gpu" and world > 1
    probe = None
    if info.get("probe_ran"):
        probe = {"pull_us": info["probe_pull_us"], "rccl_halo_us": info["probe_xchg_us"],
                 "ipc_ar_us": info["probe_alt_us"], "pull_bitwise": info["probe_pull_bitwise"],
                 "ipc_ar_close": info["probe_alt_close"], "iters_timed": info["probe_iters"],
                 "chosen": ("pull" if info.get("halo_pull") else "exchange") + "+"
                           + ("ipc" if info.get("alt_allreduce") else "rccl")}
    rehearse = bool(args.rehearse_ranks)
    return {"halo_pull": bool(info.get("halo_pull", False)),
            "halo_transport": "none" if not gpu else "in-kernel" if info.get("halo_pull") else
                              ("sdma" if rehearse else "rccl"),
            "allreduce": "none" if not gpu else "ipc" if (info.get("alt_allreduce") or rehearse) else "rccl",
            "transport_probe": probe, "rehearse_ranks": rehearse}


def _halo(v: str) -> int:
    return {"window": 0, "allgather": 1}.get(v, tri(v))


if __name__ == "__main__":
    sys.exit(main())
