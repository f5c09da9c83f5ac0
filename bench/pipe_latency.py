"""All-reduce latency sensitivity of the CG forms at one rank's share of a P-rank run.

Each all-reduce is a device-side delay (DelayComm: a one-workgroup spin of D us on the stream the
collective would run on; `fat` spins with RCCL's ~270-VGPR footprint), the rank's rows and ghost
layout are those of rank --rank of --world.  Prints one JSON line per configuration:
microseconds per iteration for each (recurrence, graph, overlap, delay, fat).

    python bench/pipe_latency.py --grid 4096 --world 8 --rank 3 --delays 0,10,20,40
"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def us_per_iter(C, spec, recurrence, delay, fat, graph, overlap, world, rank, iters, fmt, pipe_rr=0, halo_us=0.0,
                reserve_cus=0, halo_ahead=-1, halo_pull=-1, pull_proxy=0):
    o = C.CgOptions(maxit=1 << 30, tol=-1.0, check_every=1 << 30, overlap=overlap, use_graph=graph, format=fmt,
                    recurrence=recurrence)
    o.pipe_rr = pipe_rr
    o.halo_pull = halo_pull  # 1: the in-kernel halo on this rehearsal (no halo step; own lines or host memory)
    o.pull_proxy = pull_proxy
    o.reserve_cus = reserve_cus
    o.halo_ahead = halo_ahead
    comm = C.DelayComm(rank, world, delay, halo_us, fat)
    s = C.Solver(spec.native(), o, rank, world, comm)
    s.setup()
    s.reset()
    s.run_iterations(64)
    s.synchronize()
    t0 = time.perf_counter()
    s.run_iterations(iters)
    s.synchronize()
    dt = time.perf_counter() - t0
    s.finalize()
    res = s.result()
    assert res["iterations"] == 64 + iters and not res["breakdown"], res
    return 1e6 * dt / iters, s.info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", default="poisson2d")
    ap.add_argument("--grid", type=int, default=4096)
    ap.add_argument("--rows", type=int, default=1_000_000, help="randspd: global rows")
    ap.add_argument("--band", type=int, default=64)
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--delays", default="0,10,20,40")
    ap.add_argument("--recurrences", default="1,2")
    ap.add_argument("--graphs", default="1,0")
    ap.add_argument("--overlaps", default="1")
    ap.add_argument("--fat", default="0")
    ap.add_argument("--iters", type=int, default=320)
    ap.add_argument("--format", default="sellc8")
    ap.add_argument("--pipe-rr", type=int, default=0)
    ap.add_argument("--halo-us", type=float, default=0.0, help="device-side delay of each halo exchange")
    ap.add_argument("--reserve-cus", default="0", help="CgOptions.reserve_cus values (CU-masked compute stream)")
    ap.add_argument("--halo-ahead", default="-1", help="PassForm.halo_ahead values (0: interior || halo split)")
    ap.add_argument("--halo-pull", type=int, default=-1,
                    help="PassForm.halo_pull: 1 = the in-kernel halo (the pass reads the ghost lines itself, no halo "
                         "step; the rehearsal's stand-in rows), 0 = exchanged, -1 = auto (a DelayComm maps no peers: "
                         "exchanged)")
    ap.add_argument("--pull-proxy", type=int, default=0, help="with --halo-pull 1: 1 = the ghost lines in pinned host "
                                                              "memory (PCIe: a slow remote)")
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime initialised as in the other tools)

    import cuda_mpi_parallel_amd as mcg

    C = mcg.native()
    spec = (mcg.make_problem("randspd", rows=a.rows, band=a.band, density=a.density, rhs="random")
            if a.problem == "randspd" else mcg.make_problem(a.problem, n=a.grid, rhs="random"))
    ints = lambda s: [int(v) for v in s.split(",")]  # noqa: E731
    for rec, g, ov, fat, d, rc, ha in itertools.product(ints(a.recurrences), ints(a.graphs), ints(a.overlaps),
                                                        ints(a.fat), [float(v) for v in a.delays.split(",")],
                                                        ints(a.reserve_cus), ints(a.halo_ahead)):
        us, info = us_per_iter(C, spec, rec, d, bool(fat), bool(g), bool(ov), a.world, a.rank, a.iters, a.format,
                               a.pipe_rr if rec == 2 else 0, a.halo_us, rc, ha, a.halo_pull, a.pull_proxy)
        print(json.dumps({"recurrence": info["recurrence"], "graph": g, "overlap": ov, "fat": fat, "delay_us": d,
                          "us_per_iter": round(us, 2), "graph_fallbacks": info.get("graph_fallbacks"),
                          "pipe_rr": info.get("pipe_rr"), "ar_first": info.get("pipe_ar_first"),
                          "t_spmv": round(info.get("pipe_spmv_us", 0), 1), "t_ar": round(info.get("pipe_allreduce_us", 0), 1), "format": info["format"], "carry": info.get("carry"), "pmat": info.get("pmat"),
                          "problem": a.problem, "world": a.world, "rank": a.rank, "halo_us": a.halo_us,
                          "reserve_cus": rc, "halo_ahead": ha, "halo_ahead_on": info.get("halo_ahead"),
                          "halo_pull": info.get("halo_pull"), "pull_proxy": a.pull_proxy,
                          "grid": a.grid}),
              flush=True)


if __name__ == "__main__":
    main()
