#!/usr/bin/env python3
"""Copy-engine halo across PROCESSES (PeerHaloComm over IPC-mapped buffers) on one GPU: P processes
(gloo rendezvous for the handle exchange), each owning its rows of a 2-D Poisson layout, fill their
owned rows with rank-tagged values, exchange the halo `--rounds` times with new values each round,
and check every ghost row against the owner's values.  Prints one JSON line (rank 0); exit 1 on a
mismatch.  The reference has no multi-process code (CUDACG.cu:87, one device); this exercises the
north star's halo on the copy engines.

    python bench/peer_halo_check.py --world 2 [--n 256 --rounds 4]
    python bench/peer_halo_check.py --world 4 --problem scrambled   # the all-gather layout (every peer's
                                                                     # block, one copy stream per peer)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main(rank: int, a, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(a.world))
    import torch
    import torch.distributed as dist

    import cuda_mpi_parallel_amd as mcg

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=a.world)
    C = mcg.native()
    if a.problem == "scrambled":  # unstructured: the all-gather ghost layout
        spec = mcg.make_problem("randspd", rows=a.rows, band=16, density=0.5, scramble=1).native()
    else:
        spec = mcg.make_problem("poisson2d", n=a.n).native()
    L = C.make_layout(spec, a.world, rank, -1)
    assert L["allgather"] == (a.problem == "scrambled"), L["allgather"]
    ext, own, rb, nloc = L["ext_len"], L["own_off"], L["row_begin"], L["row_end"] - L["row_begin"]
    vecs = [torch.zeros(ext, dtype=torch.float64, device="cuda") for _ in range(2)]
    comm = C.PeerHaloComm(C.NullComm(rank, a.world), rank, a.world)
    comm.register_halo_buffers([v.data_ptr() for v in vecs], own, rb)
    allb = [None] * a.world
    dist.all_gather_object(allb, comm.local_handles())
    comm.attach(allb)
    stream = torch.cuda.Stream()
    bad = 0
    for rnd in range(a.rounds):
        for k, v in enumerate(vecs):  # owned rows: a function of (round, vector, global row)
            g = torch.arange(rb, rb + nloc, dtype=torch.float64, device="cuda")
            v[own:own + nloc] = 1e6 * (rnd + 1) + 1e5 * k + g
        torch.cuda.synchronize()
        dist.barrier()  # (the device flags order the copies; this barrier only makes the test's writes final)
        comm.halo_exchange_ptrs(spec, [v.data_ptr() for v in vecs], stream.cuda_stream)
        stream.synchronize()
        for _, gbegin, count in L["recvs"]:
            lo = gbegin - L["col_lo"] + L["pad"]  # LocalLayout::ext_index (partition.hpp)
            for k, v in enumerate(vecs):
                got = v[lo:lo + count].cpu()
                want = 1e6 * (rnd + 1) + 1e5 * k + torch.arange(gbegin, gbegin + count, dtype=torch.float64)
                bad += int((got != want).sum())
        dist.barrier()
    q.put((rank, bad, len(L["recvs"]), bool(L["allgather"])))
    dist.destroy_process_group()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--problem", choices=["poisson2d", "scrambled"], default="poisson2d")
    ap.add_argument("--rows", type=int, default=200000, help="scrambled: global rows")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--port", type=int, default=29531)
    ap.add_argument("--timeout", type=float, default=120.0)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=rank_main, args=(r, a, a.port, q)) for r in range(a.world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=a.timeout)
    for p in procs:  # a rank stuck on a flag wait: end it (its own process; the queue dies with it)
        if p.is_alive():
            p.kill()
            p.join()
    res = sorted(q.get(timeout=5) for _ in procs) if all(p.exitcode == 0 for p in procs) else []
    ok = bool(res) and all(b == 0 for _, b, _, _ in res) and all(p.exitcode == 0 for p in procs)
    print(json.dumps({"world": a.world, "problem": a.problem, "n": a.n, "rounds": a.rounds, "ok": ok,
                      "ranks": [{"rank": r, "mismatches": b, "recv_ranges": nr, "allgather": ag}
                                for r, b, nr, ag in res],
                      "exitcodes": [p.exitcode for p in procs]}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
