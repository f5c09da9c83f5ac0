#!/usr/bin/env python3
"""Headline benchmark: CG iterations/sec (whole node), 5-pt Poisson N=16384^2, fp64.

Metric and config come from BASELINE.json: one linear system (n = 268,435,456
rows, nnz = 1,342,111,744) solved jointly by N GPUs of one node (strong
scaling: total work fixed), matrix 1-D row-partitioned, generated on device
(synthetic — no dataset exists for this), random RHS.  A "step" is one full CG
iteration: one single-reduction pass (SpMV with Ap recomputed, the x / r / p updates
and the four dot products, reduced inside the kernel) + ONE 32-byte all-reduce of
those dot products, and at N > 1 the ghost lines (read by the pass from the
neighbours' rows, or exchanged before it: the transport probe picks at setup).
tol is disabled so every timed step does real work; the device-side iteration
counter is checked after the run.

  python bench.py                      # N=1
  python bench.py --gpus 8             # starts 8 ranks itself (one process per GPU, RCCL)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
      --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8   # same ranks under torchrun

Launch: without a torchrun environment and --gpus N > 1 (or --spawn), this process
starts the N ranks as children (cuda_mpi_parallel_amd/parallel/launch.py) BEFORE it
loads any HIP code, and exits with their status; every rank then runs exactly the
code it runs under torchrun.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

METRIC = "CG iterations/sec (whole node), 5-pt Poisson N=16384², 1/2/4/8 MI355X"
BASELINE_IT_PER_S = 65.0  # BASELINE.md "Bar to clear": reference algorithm's H100 roofline (derived; nothing published)


def aggregate(steps, ranks):
    """(iterations/s, seconds, ok) of the job from the per-rank {dt, ok, iterations} records:
    the timed region ends when the slowest rank ends, and the run is ok only if every rank is
    ok and all ranks latched the same iteration count."""
    dt = max(float(r["dt"]) for r in ranks)
    ok = all(bool(r["ok"]) for r in ranks) and len({int(r["iterations"]) for r in ranks}) == 1
    return steps / dt, dt, ok


def pass_label(info, problem):
    """The pass the timed iterations run, as the solver chose it."""
    if info.get("recurrence") == "pipelined":
        rr = info.get("pipe_rr", 0)
        return ("pipelined CG (Ghysels-Vanroose: all-reduce || SpMV)"
                + (f", residual replacement every {rr}" if rr else ""))
    if info.get("carry"):
        kind = "plane-carry" if problem == "poisson3d" or info.get("ar3_kw") else "line-carry"
        if info.get("p3"):
            kind += ", three-term (r from p_{k-1}, p_{k-2})"
        if info.get("ap_recompute"):
            kind += ", Ap recomputed"
        if info.get("lean_only"):
            kind += ", lean runs (values in scalar registers, no codes streamed)"
        if info.get("p3buf"):
            kind += ", three p buffers (no r stored)"
        if info.get("lean_mix"):
            kind += ", packed slice edges (even passes 5-6 waves/SIMD, odd passes depth 4 on their own grid)"
        return kind
    if info.get("pmat"):
        return "split (materialized p)"
    if info.get("window"):
        return "windowed"
    return "generic"


def probe_report(info, probed_ar):
    """The solver's setup-time transport probe (GpuCgSolver::probe_transport_): mean microseconds per
    iteration over the ranks of each arm it ran, what it checked, and the transports it kept."""
    r = {"iters_timed": info.get("probe_iters", 0)}
    if info.get("probe_pull_us"):
        r["pull_us"] = round(info["probe_pull_us"], 2)
    if info.get("probe_xchg_us"):
        r["rccl_halo_us"] = round(info["probe_xchg_us"], 2)
    if info.get("probe_pull_us") and info.get("probe_xchg_us"):
        r["pull_bitwise"] = bool(info.get("probe_pull_bitwise"))
    if probed_ar:
        # the first all-reduce's time = the chosen halo's arm (it ran with RCCL's all-reduce)
        r["rccl_ar_us"] = round(info["probe_pull_us"] if info.get("halo_pull") else info["probe_xchg_us"], 2)
        r["ipc_ar_us"] = round(info.get("probe_alt_us", 0.0), 2)
        r["ipc_ar_close"] = bool(info.get("probe_alt_close"))
        if info.get("probe_alt_timeout"):
            r["ipc_ar_timeout"] = True
    r["chosen"] = ("pull" if info.get("halo_pull") else "exchange") + "+" + ("ipc" if info.get("alt_allreduce") else "rccl")
    return r


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--grid", type=int, default=16384, help="grid edge N (N^2 rows for poisson2d)")
    ap.add_argument("--problem", default="poisson2d", choices=["poisson2d", "poisson3d", "randspd"])
    ap.add_argument("--rows", type=int, default=100_000_000, help="randspd: global rows")
    ap.add_argument("--band", type=int, default=4096, help="randspd: half bandwidth")
    ap.add_argument("--density", type=float, default=0.16, help="randspd: candidate-pair density")
    ap.add_argument("--spread", type=int, default=0,
                    help="randspd: > 0 = candidate offsets over [1, spread] (wide multi-diagonal; the all-gather path)")
    ap.add_argument("--scramble", type=int, default=0,
                    help="randspd: 1 = P^T A P with a seeded random permutation P (genuinely irregular sparsity)")
    ap.add_argument("--coef", type=int, default=0,
                    help="poisson2d/3d: 1 = variable coefficients (seeded random conductivity field; not the headline)")
    ap.add_argument("--format", default="sellc8", choices=["csr", "sell", "sell16", "sellc8"],
                    help="sparse storage: CSR, SELL-64, SELL-64/d16 (16-bit column offsets) or SELL-64/c8 "
                         "(one-byte (value, offset) dictionary codes; default, falls back to d16)")
    ap.add_argument("--recurrence", type=int, default=-1,
                    help="0 two-reduction, 1 single-reduction, 2 pipelined (Ghysels-Vanroose), -1 auto")
    ap.add_argument("--pipe-rr", type=int, default=0,
                    help="pipelined CG: residual replacement every K iterations (0 = off)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph", action="store_true", help="(default since r2; kept for old command lines)")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--blocks-per-cu", type=int, default=0, help="SpMV grid; 0 = auto")
    ap.add_argument("--no-verify", action="store_true", help="skip the true-residual check ||b-Ax|| after the run")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="experiment: set a native CgOptions field (e.g. halo_pull=0, placement_tries=1)")
    ap.add_argument("--phases", type=int, default=10,
                    help="after the timed region: N more iterations with per-phase hipEvent timing (diagnostic, "
                         "reported under check.phase_us of rank 0 and check.phase_us_max over ranks; 0 = off)")
    ap.add_argument("--comm", default="single", choices=["dual", "single"],
                    help="single (default): one RCCL communicator, every collective in one stream order on the "
                         "compute stream; dual: reduce + halo communicators, the halo on the side stream next to the "
                         "all-reduce (profiles/r3_priced_shares.md: 1-6 %% slower at P = 8 shares, two "
                         "communicators in flight at once)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the RCCL collectives also with one rank (1-rank communicator): the N > 1 code path")
    ap.add_argument("--halo-transport", default="auto", choices=["auto", "rccl", "sdma"],
                    help="auto (N > 1): the neighbours' buffers mapped through IPC (PeerHaloComm) for the lean "
                         "carries' in-kernel halo (halo_pull: checked at setup, off again if any rank cannot map or "
                         "reads a wrong row), every remaining halo exchange and the all-reduce on RCCL; rccl: no "
                         "mapping; sdma: the halo exchanges on copy engines (flags by stream memory operations)")
    ap.add_argument("--allreduce", default="auto", choices=["auto", "rccl", "ipc"],
                    help="auto (N > 1 on N GPUs): every rank's IPC all-reduce mailbox mapped next to RCCL, and the "
                         "solver's transport probe times both at setup and keeps the faster correct one (check."
                         "transport_probe); rccl: RCCL only; ipc: the 32-byte all-reduce through IPC-mapped mailboxes "
                         "(PeerHaloComm + csrc/gpu/ipc_allreduce.hip, no RCCL; implies the peer-mapped halo).  With "
                         "--rehearse-ranks the P processes on one GPU then run the real P-rank recurrence")
    ap.add_argument("--delay-comm", default="",
                    help="with --sim-world: AR_US,HALO_US[,copy|fat] -- every all-reduce / halo (or all-gather) exchange "
                         "of the rehearsed rank costs a device-side delay of that many microseconds (DelayComm) "
                         "instead of nothing (NullComm); 'copy': the halo is real copy-engine traffic of the "
                         "layout's message sizes (a CU-free transport's timing); 'fat': the delays spin with RCCL's "
                         "~270 VGPRs per wave (they cannot start beside a resident kernel)")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="timing rehearsal: run rank --sim-rank of a P-rank job alone on this GPU (its rows, "
                         "ghost layout, interior/boundary launches, graphs) with collectives that move nothing")
    ap.add_argument("--sim-rank", type=int, default=0)
    ap.add_argument("--watchdog", type=float, default=600.0,
                    help="seconds a host wait may go without progress before the run fails and RCCL is aborted "
                         "(a hung collective ends the job with a message instead of hanging; 0 = unbounded)")
    ap.add_argument("--rehearse-ranks", action="store_true",
                    help="multi-process rehearsal on ONE GPU: --gpus P ranks (spawned, or under torchrun) all on "
                         "device 0 with collectives that move nothing (NullComm), but the real gloo rendezvous, "
                         "barriers and all_gather_object aggregation of the P-rank bench")
    ap.add_argument("--spawn", action="store_true",
                    help="start the rank(s) as child processes even for --gpus 1 (the --gpus N > 1 launch route)")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    from cuda_mpi_parallel_amd.parallel import launch

    # (a) --gpus N without torchrun: start the ranks and exit with their status.  Only the
    # parent decides; a child (WORLD_SIZE set) always runs as a rank.
    rc = launch.launch_or_none(args.gpus, [a for a in argv if a != "--spawn"], force_spawn=args.spawn,
                               script=os.path.abspath(__file__), share_device=args.rehearse_ranks)
    if rc is not None:
        return rc
    return run_rank(args)


def run_rank(args) -> int:
    # stdout carries exactly one JSON line: RCCL prints a version banner on stdout at communicator
    # init, so fd 1 points at stderr until the result is printed
    out_fd = os.dup(1)
    os.dup2(2, 1)
    try:
        return _run_rank(args, out_fd)
    finally:
        sys.stdout.flush()
        os.dup2(out_fd, 1)
        os.close(out_fd)


def _run_rank(args, out_fd) -> int:
    import torch
    import torch.distributed as dist

    import cuda_mpi_parallel_amd as mcg
    from cuda_mpi_parallel_amd.parallel import dist as pdist
    from cuda_mpi_parallel_amd.parallel import launch

    env = pdist.dist_env()
    n_gpus = env.world
    route = "spawn" if os.environ.get(launch.CHILD_FLAG) else ("torchrun" if launch.under_launcher() else "single")
    # no user-buffer registration while capturing RCCL calls into graphs (buffers are few and
    # small; registration would add an IPC-handle path the solver does not need)
    os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
    rehearse = args.rehearse_ranks and env.world > 1
    if rehearse:  # every rank on device 0 (RCCL refuses two ranks on one GPU: collectives move nothing)
        torch.cuda.set_device(0)
    else:
        pdist.set_device(env)
    if env.world > 1:
        pdist.init_process_group(env, backend="gloo")
    comm = mcg.native().NullComm(env.rank, env.world) if rehearse else pdist.bootstrap_comm(env, force=args.force_comm, mode=args.comm)
    sim = args.sim_world > 1 and env.world == 1
    if sim:  # per-rank timing rehearsal (not a P-rank solve: see --sim-world)
        if args.delay_comm:
            f = args.delay_comm.split(",")
            comm = mcg.native().DelayComm(args.sim_rank, args.sim_world, float(f[0]), float(f[1]), "fat" in f[2:],
                                          "copy" in f[2:])
        else:
            comm = mcg.native().NullComm(args.sim_rank, args.sim_world)

    if args.problem == "randspd":
        spec = mcg.make_problem("randspd", rows=args.rows, band=args.band, density=args.density, spread=args.spread,
                                scramble=args.scramble, rhs="random")
    else:
        spec = mcg.make_problem(args.problem, n=args.grid, rhs="random", coef=args.coef)
    C = mcg.native()
    # hipGraph replay of 32-iteration blocks at every N: at N > 1 the RCCL all-reduce and the halo
    # send/recv (forked onto the side stream and joined by events) are captured with the kernels,
    # so the host enqueues one graph per 32 iterations; a failed capture falls back to eager
    use_graph = not args.no_graph
    opts = C.CgOptions(maxit=1 << 30, tol=-1.0, check_every=1 << 30, overlap=not args.no_overlap,
                       use_graph=use_graph, force_comm=args.force_comm, format=args.format,
                       blocks_per_cu=args.blocks_per_cu, recurrence=args.recurrence)
    opts.watchdog_seconds = args.watchdog
    opts.pipe_rr = args.pipe_rr
    for kv in args.set:
        k, v = kv.split("=", 1)
        if not hasattr(opts, k):
            raise SystemExit(f"bench.py: unknown option {k!r}")
        setattr(opts, k, type(getattr(opts, k))(v))
    t_setup = time.perf_counter()
    ipc_ar = args.allreduce == "ipc" and comm is not None and not sim
    sdma = (args.halo_transport == "sdma" or ipc_ar) and comm is not None and not sim
    # auto: the mapping for the in-kernel halo, the exchanges on the inner communicator (a rehearsal's
    # inner moves nothing: there only the real P-rank form, ipc_ar, takes the copy-engine exchanges)
    mapped = (sdma or args.halo_transport == "auto") and comm is not None and not sim and env.world > 1
    # --allreduce auto: the IPC mailboxes mapped but not selected, so the solver's transport probe (first
    # reset) times them against RCCL's all-reduce and keeps the faster one that reproduces RCCL's sums
    probe_ar = args.allreduce == "auto" and mapped and not rehearse
    base_comm = comm  # RCCL's (or the rehearsal's) communicator: the count, the all-reduce
    if mapped:
        comm = pdist.peer_halo(comm, env, ipc_allreduce=ipc_ar or probe_ar, halo_via_inner=not sdma, tolerant=probe_ar)
        if probe_ar:
            comm.ipc_allreduce = False
    real = not sim and (not rehearse or ipc_ar)  # a real P-rank solve (its residual must track)
    solver = (C.Solver(spec.native(), opts, args.sim_rank, args.sim_world, comm) if sim
              else C.Solver(spec.native(), opts, env.rank, env.world, comm))
    solver.setup()
    if mapped:
        pdist.attach_peer_halo(comm, env, tolerant=not sdma)
    solver.reset()
    setup_s = time.perf_counter() - t_setup

    def barrier():
        if env.world > 1:
            dist.barrier()

    solver.run_iterations(args.warmup)
    solver.synchronize()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    solver.run_iterations(args.steps)
    solver.synchronize()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0


    phases = None
    if args.phases > 0 and solver.info["recurrence"] == "single-reduction":
        phases = solver.phase_profile(args.phases)  # untimed diagnostics: per-phase mean microseconds
        phases = {k: round(v, 2) for k, v in phases.items()}
    n_extra = args.phases if phases is not None else 0
    solver.finalize()  # untimed: completes x_m (the single-reduction form pairs x updates) and latches
    res = solver.result()
    ok = res["iterations"] == args.warmup + args.steps + n_extra and not res["breakdown"] and math.isfinite(res["rnorm"])
    extra = {}
    if not args.no_verify:
        # the recurrence residual must track the true residual ||b - A x|| (catches a kernel
        # that does less work than claimed: its residual would drift from the truth by orders
        # of magnitude).  Over the bench's few hundred iterations the two agree to ~1e-15
        # relative (fp64 round-off only), so the guard is tight.  Once ||b - A x|| is 9 orders
        # below ||b|| the true residual stagnates at fp64's attainable accuracy while the
        # recurrence keeps falling (both CG forms, e.g. 512^3 after 2000 iterations:
        # profiles/r2s6_long_runs.md); a solve that converged that far has done its work
        tr = solver.true_residual_norm()
        rr0 = torch.tensor([float(res.get("rr0_local", 0.0))], dtype=torch.float64)
        if env.world > 1 and not sim:
            dist.all_reduce(rr0)  # gloo (host): every rank's b.b
        bnorm = math.sqrt(max(float(rr0.item()), 0.0))
        extra["true_rnorm"] = tr
        extra["true_gap_rel"] = abs(tr - res["rnorm"]) / max(tr, 1e-300)
        extra["true_rel_to_b"] = tr / max(bnorm, 1e-300)
        tracks = abs(tr - res["rnorm"]) <= 1e-8 * max(tr, 1e-300) + 1e-12
        ok = ok and (not real or tracks or tr <= 1e-9 * bnorm)
    info = solver.info
    # whole-job result: the slowest rank's clock, every rank ok and latched at the same count
    mine = {"dt": dt, "ok": bool(ok), "iterations": int(res["iterations"])}
    ranks = [mine]
    if env.world > 1:
        ranks = [None] * env.world
        dist.all_gather_object(ranks, mine)
    value, dt, ok = aggregate(args.steps, ranks)
    nnz = spec.nnz
    if nnz is None:  # randspd: no closed form; sum the ranks' generated counts
        t = torch.tensor([info["nnz_local"]], dtype=torch.int64)
        if env.world > 1:
            dist.all_reduce(t)
        nnz = int(t.item())
    headline = args.problem == "poisson2d" and args.grid == 16384 and not sim and not rehearse and not args.coef
    if phases is not None:
        extra["phase_us"] = phases
        if env.world > 1:  # slowest rank per phase
            keys = sorted(phases)
            t = torch.tensor([phases[k] for k in keys], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            extra["phase_us_max"] = {k: round(float(v), 2) for k, v in zip(keys, t.tolist())}
    model = (f"randspd_rows{args.rows}_band{args.band}_q{args.density}" + (f"_spread{args.spread}" if args.spread else "")
             + ("_scrambled" if args.scramble else "") if args.problem == "randspd" else
             f"{args.problem}_N{args.grid}" + ("_varcoef" if args.coef else ""))
    if env.rank == 0:
        line = json.dumps({
            "metric": METRIC if headline else (
                "per-rank iterations/sec, timing rehearsal of rank %d of %d (collectives move nothing), %s"
                % (args.sim_rank, args.sim_world, model) if sim else
                "rehearsal: %d ranks on ONE GPU (IPC all-reduce + peer-mapped halo: the real %d-rank recurrence), %s"
                % (env.world, env.world, model) if rehearse and ipc_ar else
                "rehearsal: %d ranks on ONE GPU (collectives move nothing; rendezvous / barriers / aggregation real), %s"
                % (env.world, model) if rehearse else "CG iterations/sec (whole node), %s" % model),
            "value": round(value, 4),
            "unit": "iterations/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / BASELINE_IT_PER_S, 4) if headline else None,
            "dtype": "fp64",
            "data": "synthetic (on-device generated %s matrix, random RHS)" % {
                "poisson2d": "5-pt Poisson" + (" (variable coefficients)" if args.coef else ""),
                "poisson3d": "7-pt Poisson" + (" (variable coefficients)" if args.coef else ""),
                "randspd": "random SPD " + ("scrambled P^T A P (irregular)" if args.scramble else
                                            "wide multi-diagonal" if args.spread else "banded")}[args.problem],
            "config": {
                "model": model,
                "problem": args.problem,
                "N": args.grid,
                "rows": spec.n_rows,
                "nnz": nnz,
                "global_batch": 1,
                "seq_len": spec.n_rows,
                "parallelism": (f"sim-rank{args.sim_rank}-of-{args.sim_world}"
                                + (f"-delaycomm{args.delay_comm.replace(',', '-')}us" if args.delay_comm else "") if sim else
                                f"rehearse-rowpart{n_gpus}-one-gpu" if rehearse else f"rowpart{n_gpus}"),
                # storage the timed pass streams (the carries read SELL-64/dia4 codes; their lean runs
                # only the per-slice pattern words of uniform slices)
                "format": (("sell64-dia4, uniform-slice patterns" if info.get("lean_only") else "sell64-dia4")
                           if info.get("dia4") else
                           "sell64-diav (each row's own values streamed)" if info.get("diav") else
                           info["format"]),
                "recurrence": info["recurrence"],
                "pass": pass_label(info, args.problem),
                **({"ghosts": ("allgather || own-block SpMV half" if info.get("ag_overlap") else "allgather")
                    if info.get("allgather") else ("window, read in-kernel from the neighbours' rows (halo_pull)"
                                                   if info.get("halo_pull") else
                                                   "window, exchanged ahead || all-reduce" if info.get("halo_ahead")
                                                   else "window")} if (n_gpus > 1 or sim) else {}),
                "hipgraph": bool(info.get("graphs", use_graph)) and info.get("graph_fallbacks", 0) == 0,
                "fused_reduce": info.get("fused_reduce", False),
                "halo_overlap": (not args.no_overlap) and n_gpus > 1 and args.comm == "dual",
                "comm": args.comm,
                **({"halo_transport": ("in-kernel (the pass reads the IPC-mapped neighbour rows)" if info.get("halo_pull")
                                       else "sdma (copy engines, IPC)" if sdma else "rccl (mapping unused)"),
                    "allreduce": "ipc (mapped mailboxes)" if (ipc_ar or info.get("alt_allreduce")) else "rccl"}
                   if mapped else {}),
                "launch": route,
                **({"reserve_cus": opts.reserve_cus} if opts.reserve_cus else {}),
            },
            "check": {"device_iterations": res["iterations"], "rnorm": res["rnorm"], "ok": ok,
                      "comm_world": base_comm.count if (comm is not None and not sim and not rehearse) else 1,
                      "rccl": mcg.native().rccl_info(),
                      "graph_fallbacks": info.get("graph_fallbacks", 0),
                      "setup_s": round(setup_s, 3), "placement_sets": info.get("placement_sets"),
                      "placement_gain": round(info.get("placement_gain", 1.0), 4),
                      # the probe's spread: two passes' time on its best and worst placement (setup)
                      "placement_best_ms": round(info.get("placement_best_ms", 0.0), 4),
                      "placement_worst_ms": round(info.get("placement_worst_ms", 0.0), 4),
                      "placement_lead_trial": info.get("placement_lead_trial"),
                      "dia_uniform": round(info.get("dia_uniform", 0.0), 4), "lean_only": info.get("lean_only", False),
                      "halo_pull": info.get("halo_pull", False),
                      **({"transport_probe": probe_report(info, probe_ar)} if info.get("probe_ran") else {}),
                      **({"ag_local_frac": round(info["ag_local_frac"], 4)} if info.get("ag_overlap") else {}),
                      "model_gb_per_iter_rank0": round(info["bytes_per_iter_model"] / 1e9, 3),
                      "model_tb_per_s_rank0": round(info["bytes_per_iter_model"] * value / 1e12, 3),
                      "device_gb_rank0": round(info["device_bytes"] / 1e9, 2), **extra},
        })
        sys.stdout.flush()
        os.write(out_fd, (line + "\n").encode())
    if env.world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
