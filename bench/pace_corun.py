#!/usr/bin/env python3
"""What the L2-segment tile pacing costs when another kernel shares the GPU.

The tiles SpMV (csrc/gpu/cg_tiles.hip) paces its workgroups per column segment and assumes they are
all resident; a workgroup that waits longer than the cap (~1 ms) gives up pacing for the rest of the
launch.  At P > 1 an RCCL kernel (an all-gather in flight, ~270 VGPRs per wave) can hold CUs while
the SpMV runs.  This probe times the split pass alone and then with `--spinners` one-workgroup spins
of RCCL's register footprint (`fat`) or a thin one running on a side stream for the whole timed
region, and prints one JSON line.

    python bench/pace_corun.py [--rows 12500000 --band 410] [--spinners 1 8 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--band", type=int, default=410)
    ap.add_argument("--world", type=int, default=8, help="rehearse rank --rank of this many (NullComm)")
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--spinners", type=int, nargs="*", default=[1, 8, 32])
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    a = ap.parse_args()
    import torch

    import cuda_mpi_parallel_amd as mcg

    torch.cuda.set_device(0)
    C = mcg.native()
    spec = mcg.make_problem("randspd", rows=a.rows, band=a.band, density=1.0, scramble=1, rhs="random")
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, check_every=1 << 30, format="sellc8", recurrence=1)
    for kv in a.set:
        k, v = kv.split("=", 1)
        setattr(o, k, type(getattr(o, k))(v))
    s = C.Solver(spec.native(), o, a.rank, a.world, C.NullComm(a.rank, a.world))
    s.setup()
    s.reset()
    s.run_iterations(2)
    s.synchronize()
    side = torch.cuda.Stream(priority=-1)
    sink = torch.zeros(64, dtype=torch.float64, device="cuda")

    def timed():
        t0 = time.perf_counter()
        s.run_iterations(a.iters)
        s.synchronize()
        return 1e3 * (time.perf_counter() - t0) / a.iters

    out = {"rows": a.rows, "band": a.band, "share": f"rank{a.rank}-of-{a.world}", "tiles": s.info.get("tiles"),
           "tile_segments": s.info.get("tile_segments"), "alone_ms": round(timed(), 3)}
    for fat in (True, False):
        for n in a.spinners:
            # spins that outlast the timed region: launched first, then the iterations queue behind them
            C.kernels.spin(sink.data_ptr(), 1e3 * (a.iters + 4) * out["alone_ms"] * 2.0, fat, n, side.cuda_stream)
            time.sleep(0.002)
            out[f"{'fat' if fat else 'thin'}{n}_ms"] = round(timed(), 3)
            torch.cuda.synchronize()
    out["alone_again_ms"] = round(timed(), 3)
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
