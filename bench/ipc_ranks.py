#!/usr/bin/env python3
"""The real P-rank recurrence across PROCESSES on one GPU: P processes (gloo rendezvous for the IPC
handle exchange) each run their rows of the CG solver with the IPC all-reduce (PeerHaloComm mailboxes,
csrc/gpu/ipc_allreduce.hip) and the peer-mapped halo -- the in-kernel halo (halo_pull: the lean pass
reads the neighbours' rows) or the copy-engine pulls (halo_pull 0) -- for a fixed iteration count, in
32-iteration hipGraphs.  The parent then solves the same system with one rank and compares the
residual norm and x.  The reference's two global reductions (CUDACG.cu:304, :328) are what the
all-reduce carries; RCCL refuses two ranks on one GPU, so this is the only cross-process P-rank solve
the one-GPU pool can run.  Prints one JSON line; exit 1 when a rank fails or the gap is too large.

    python bench/ipc_ranks.py --world 2 [--problem poisson2d --n 1024 --iters 40 --halo-pull -1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _opts(C, a):
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, check_every=1 << 30, format="sellc8", recurrence=a.recurrence)
    o.halo_pull = a.halo_pull
    # the transport probe (first reset) runs the pulled and the exchanged arm; which it keeps is pinned
    # here (by default the pull, as before the probe) so the test knows the path
    o.probe_pick_halo = a.probe_pick
    o.transport_probe = a.transport_probe
    o.pipe_rr = a.pipe_rr
    o.use_graph = not a.no_graph
    o.overlap = bool(a.overlap)
    o.watchdog_seconds = 60.0
    return o


def _spec(mcg, a):
    if a.problem == "scrambled":  # irregular: the all-gather layout, the split pass (single exchanged p)
        return mcg.make_problem("randspd", rows=a.rows, band=16, density=0.5, scramble=1, rhs="random").native()
    return mcg.make_problem(a.problem, n=a.n, rhs="random", coef=a.coef).native()


def log(rank, msg):
    import time

    print(f"[rank {rank}] {time.strftime('%X')} {msg}", file=sys.stderr, flush=True)


def rank_main(rank: int, a, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(a.world))
    import torch
    import torch.distributed as dist

    import cuda_mpi_parallel_amd as mcg
    from cuda_mpi_parallel_amd.parallel import dist as pdist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=a.world)
    env = pdist.DistEnv(rank=rank, world=a.world, local_rank=0)
    C = mcg.native()
    comm = pdist.peer_halo(C.NullComm(rank, a.world), env, ipc_allreduce=True)
    comm.ar_budget_seconds = a.budget
    log(rank, "mailboxes mapped")
    s = C.Solver(_spec(mcg, a), _opts(C, a), rank, a.world, comm)
    s.setup()
    log(rank, "setup done")
    pdist.attach_peer_halo(comm, env)
    s.reset()
    log(rank, "reset done")
    s.run_iterations(a.iters)
    s.synchronize()
    log(rank, "iterations done")
    s.finalize()
    res = s.result()
    log(rank, "finalized")
    x = np.asarray(s.x_local())
    tr = s.true_residual_norm()
    log(rank, "true residual done")
    info = s.info
    q.put((rank, float(res["rnorm"]), int(res["iterations"]), x.tobytes(), float(tr),
           bool(info.get("halo_pull")), bool(info.get("lean_only")), int(info.get("graph_fallbacks", 0)),
           bool(info.get("graphs")), {k: info.get(k) for k in ("probe_ran", "probe_pull_us", "probe_xchg_us",
                                                                 "probe_pull_bitwise", "probe_iters")}))
    dist.barrier()
    dist.destroy_process_group()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--problem", choices=["poisson2d", "poisson3d", "scrambled"], default="poisson2d")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=200000, help="scrambled: global rows")
    ap.add_argument("--recurrence", type=int, default=1, help="1 single-reduction, 2 pipelined")
    ap.add_argument("--pipe-rr", type=int, default=0)
    ap.add_argument("--coef", type=int, default=0)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--halo-pull", type=int, default=-1)
    ap.add_argument("--probe-pick", type=int, default=1, help="transport probe: keep the pull (1) / exchange (0) / "
                                                              "the faster (-1)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--transport-probe", type=int, default=-1, help="0: no transport probe at the first reset")
    ap.add_argument("--overlap", type=int, default=1, help="0: the halo in the pass's stream order (no halo_ahead)")
    ap.add_argument("--tol", type=float, default=1e-13, help="relative gap allowed against one rank")
    ap.add_argument("--port", type=int, default=29541)
    ap.add_argument("--timeout", type=float, default=180.0)
    ap.add_argument("--budget", type=float, default=60.0, help="IPC all-reduce: seconds a peer may be late")
    a = ap.parse_args()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=rank_main, args=(r, a, a.port, q)) for r in range(a.world)]
    for p in procs:
        p.start()
    import time

    import queue

    # read the results before joining: a child that put a large x on the queue exits only once the
    # queue's feeder thread has handed it over
    t_end = time.time() + a.timeout
    res = []
    try:
        for _ in procs:
            res.append(q.get(timeout=max(1.0, t_end - time.time())))
    except queue.Empty:
        res = []
    for p in procs:
        p.join(timeout=max(1.0, t_end - time.time()))
    for p in procs:  # a rank stuck (its all-reduce times out on its own budget): end it
        if p.is_alive():
            p.kill()
    res = sorted(res) if len(res) == len(procs) and all(p.exitcode == 0 for p in procs) else []
    out = {"world": a.world, "problem": a.problem, "n": a.n, "coef": a.coef, "iters": a.iters,
           "recurrence": a.recurrence, "pipe_rr": a.pipe_rr,
           "halo_pull_opt": a.halo_pull, "graphs": not a.no_graph, "exitcodes": [p.exitcode for p in procs]}
    ok = bool(res) and all(p.exitcode == 0 for p in procs)
    if ok:
        import cuda_mpi_parallel_amd as mcg

        C = mcg.native()
        one = C.run_local_ranks(_spec(mcg, a), _opts(C, a), 1, a.iters, True)
        r1 = one["ranks"][0]["rnorm"]
        x1 = np.asarray(one["x"])
        xp = np.concatenate([np.frombuffer(r[3], dtype=np.float64) for r in res])
        gap_r = max(abs(r[1] - r1) / r1 for r in res)
        gap_x = float(np.linalg.norm(xp - x1) / np.linalg.norm(x1))
        out.update(rnorm_1=r1, rnorm_p=res[0][1], gap_rnorm=gap_r, gap_x=gap_x,
                   true_gap=max(abs(r[4] - r[1]) / r[4] for r in res),
                   ranks=[{"rank": r[0], "iterations": r[2], "halo_pull": r[5], "lean_only": r[6],
                           "graph_fallbacks": r[7], "graphs": r[8], **r[9]} for r in res])
        ok = (gap_r <= a.tol and gap_x <= 10 * a.tol and all(r[2] == a.iters for r in res)
              and len({r[1] for r in res}) == 1)
    out["ok"] = ok
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
