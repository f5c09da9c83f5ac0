#!/usr/bin/env python3
"""Can a halo collective run WHILE the CG pass occupies the GPU?  (one MI355X, no peers needed)

At P > 1 the halo send/recv of an iteration runs on the side stream next to the interior pass.
RCCL moves p2p data with kernels, so the overlap only exists if its workgroups find room on the
CUs while the pass is resident.  The line-carry pass is a fully resident grid (4 blocks/CU, ~120
VGPRs, every wave walks a long run of grid lines and retires only at the end), so it may leave no
room.  This probe measures it on one GPU: a 1-rank RCCL communicator's grouped send/recv to itself
(the same Comm::sendrecv the halo uses, a 393 KB message = one 16384-row {r, Ap} + p ghost line)
and a small elementwise torch kernel, timed on a high-priority stream
  (a) alone, and
  (b) enqueued right after several solver iterations are queued on the solver's stream.
If (b) takes about as long as (a), the collective overlaps the pass; if it takes about a pass
(~3 ms), it waited for the pass to drain.

Controls (r3): `spin_fat` = one 256-thread workgroup spinning 20 us with ~270
VGPRs per wave live (RCCL's kernels' footprint) and no RCCL; `spin_thin` = the same with a few
VGPRs.  If spin_fat waits like RCCL and spin_thin does not, the register file is the blocker; if
spin_fat starts at once, something RCCL-specific is (its queue / the loopback path).  Run under
`rocprofv3 --kernel-trace` the dispatches' queue ids and start / end stamps show which queue each
kernel used and when it started relative to the pass (bench/corun_trace.py).

  python bench/corun_probe.py [--grid 16384] [--set carry_blocks_per_cu=3 ...]
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
    ap.add_argument("--grid", type=int, default=16384)
    ap.add_argument("--problem", default="poisson2d")
    ap.add_argument("--iters", type=int, default=8, help="solver iterations queued ahead of each probe")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--doubles", type=int, default=3 * 16384, help="message size (doubles)")
    ap.add_argument("--graph", type=int, default=1, help="solver iterations as hipGraphs (1) or eager (0)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE", help="extra CgOptions")
    ap.add_argument("--copy-kib", type=int, action="append", default=[],
                    help="r4: also time two side-stream hipMemcpyAsync copies of this many KiB each, with the "
                         "copy engine (hipMemcpyDeviceToDeviceNoCU) and with the default (blit-kernel) path")
    ap.add_argument("--kinds", default="rccl,rccl_graph,torch_add,spin_fat,spin_thin")
    a = ap.parse_args()

    import torch

    import cuda_mpi_parallel_amd as mcg

    torch.cuda.set_device(0)
    C = mcg.native()
    spec = mcg.make_problem(a.problem, n=a.grid)
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1)
    o.use_graph = bool(a.graph)
    for kv in a.set:
        k, v = kv.split("=", 1)
        setattr(o, k, type(getattr(o, k))(v))
    s = C.Solver(spec.native(), o)
    s.setup()
    s.reset()
    s.run_iterations(4)
    s.synchronize()
    comm = C.Comm(0, 1, C.unique_id(), C.unique_id())
    n = a.doubles
    src = torch.rand(n, dtype=torch.float64, device="cuda")
    dst = torch.zeros_like(src)
    side = torch.cuda.Stream(priority=-1)
    spin_out = torch.zeros(64, dtype=torch.float64, device="cuda")
    # two ghost-sized copies (lo / hi halo) per probe: the CU-free transport candidate
    cmax = max(a.copy_kib or [0]) * 1024
    csrc = torch.rand(max(1, 2 * cmax // 8), dtype=torch.float64, device="cuda")
    cdst = torch.zeros_like(csrc)

    # the same send/recv captured into a graph on the side stream (how the halo runs at P > 1):
    # separates a host-side wait inside the RCCL call from a device-side wait for CUs
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        comm.sendrecv_ptr(src.data_ptr(), 0, dst.data_ptr(), 0, n, side.cuda_stream)
    torch.cuda.synchronize()
    host_us = {}

    def probe(kind):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            e0.record(side)
            h0 = time.perf_counter()
            if kind == "rccl":
                comm.sendrecv_ptr(src.data_ptr(), 0, dst.data_ptr(), 0, n, side.cuda_stream)
            elif kind == "rccl_graph":
                g.replay()
            elif kind.startswith("copy_"):
                _, eng, kib = kind.split("_")
                nb = int(kib) * 1024
                k = 1024 if eng == "nocu" else 3
                for h in range(2):
                    C.kernels.memcpy_async(cdst.data_ptr() + h * nb, csrc.data_ptr() + h * nb, nb, k, side.cuda_stream)
            elif kind in ("spin_fat", "spin_thin"):
                C.kernels.spin(spin_out.data_ptr(), 20.0, kind == "spin_fat", 1, side.cuda_stream)
            else:
                torch.add(src, 1.0, out=dst)
            host_us.setdefault(kind, []).append(round((time.perf_counter() - h0) * 1e6, 1))
            e1.record(side)
        return e0, e1

    # solver pass time (for scale)
    t0 = time.perf_counter()
    s.run_iterations(16)
    s.synchronize()
    pass_ms = (time.perf_counter() - t0) * 1e3 / 16

    out = {"problem": a.problem, "grid": a.grid, "pass_ms": round(pass_ms, 3), "info": {k: s.info[k] for k in ("carry", "format")}}
    kinds = [k for k in a.kinds.split(",") if k]
    for kib in a.copy_kib:
        kinds += [f"copy_nocu_{kib}", f"copy_blit_{kib}"]
    for kind in kinds:
        alone, busy = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = probe(kind)
            torch.cuda.synchronize()
            alone.append(e0.elapsed_time(e1) * 1e3)
            s.run_iterations(a.iters)  # the pass is now queued / running on the solver's stream
            time.sleep(0.0005)         # let the first pass start and fill the CUs
            e0, e1 = probe(kind)
            s.synchronize()
            torch.cuda.synchronize()
            busy.append(e0.elapsed_time(e1) * 1e3)
        out[kind] = {"alone_us": [round(v, 1) for v in alone], "with_pass_us": [round(v, 1) for v in busy],
                     "host_call_us": host_us.get(kind, [])[1::2]}
    comm.check_async()
    print(json.dumps(out), flush=True)
    # a graph holding captured RCCL work must go before its communicator; even then the
    # interpreter's teardown of both has been seen to hang, so leave without it
    del g
    torch.cuda.synchronize()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)


if __name__ == "__main__":
    sys.exit(main())
