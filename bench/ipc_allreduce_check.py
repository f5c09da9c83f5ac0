#!/usr/bin/env python3
"""The IPC all-reduce alone (PeerHaloComm mailboxes, csrc/gpu/ipc_allreduce.hip) across PROCESSES on one
GPU: P processes sum rank-tagged values `--calls` times (eager and from a captured hipGraph) and check
every sum against the closed form; a rank whose peer never arrives sees the error word after the
budget (--budget seconds) instead of hanging.  Prints progress lines (stderr) and one JSON line.
Also times the call (microseconds, eager back-to-back) as the latency candidate against RCCL's 32-byte
all-reduce.  The reference's two global dot products (CUDACG.cu:304, :328) are what it carries.

    python bench/ipc_allreduce_check.py --world 2 [--calls 200 --budget 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def log(rank, msg):
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
    stream = torch.cuda.Stream()
    buf = torch.zeros(4, dtype=torch.float64, device="cuda")
    bad = 0
    t_us = 0.0
    with torch.cuda.stream(stream):
        for c in range(a.calls):
            buf.copy_(torch.tensor([rank + 1.0, c * 1.0, (rank + 1) * 0.5, 1.0], dtype=torch.float64))
            comm.allreduce_ptr(buf.data_ptr(), 4, stream.cuda_stream)
            got = buf.cpu().tolist()
            P = a.world
            want = [P * (P + 1) / 2, c * 1.0 * P, P * (P + 1) / 4, 1.0 * P]
            bad += int(got != want)
            if c == 0:
                log(rank, f"first call ok={got == want} got={got}")
        log(rank, f"{a.calls} eager calls, mismatches {bad}")
        # timing: back-to-back calls (no host sync in between)
        dist.barrier()
        stream.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            comm.allreduce_ptr(buf.data_ptr(), 4, stream.cuda_stream)
        stream.synchronize()
        t_us = 1e6 * (time.perf_counter() - t0) / a.calls
        log(rank, f"back-to-back {t_us:.2f} us per call")
        # captured: the device-side call counter replays correctly
        buf.fill_(1.0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(3):
                comm.allreduce_ptr(buf.data_ptr(), 4, stream.cuda_stream)
        dist.barrier()
        buf.fill_(1.0)
        g.replay()
        g.replay()
        stream.synchronize()
        gv = buf.cpu().tolist()
        want_g = float(a.world) ** 6
        gbad = int(any(v != want_g for v in gv))
        log(rank, f"graph replays {gv} (want {want_g})")
    try:
        comm.check_async()
        err = 0
    except Exception as e:  # noqa: BLE001
        log(rank, f"error word set: {e}")
        err = 1
    q.put((rank, bad, gbad, err, t_us))
    dist.barrier()
    dist.destroy_process_group()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--budget", type=float, default=10.0)
    ap.add_argument("--port", type=int, default=29551)
    ap.add_argument("--timeout", type=float, default=90.0)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=rank_main, args=(r, a, a.port, q)) for r in range(a.world)]
    for p in procs:
        p.start()
    t_end = time.time() + a.timeout
    for p in procs:
        p.join(timeout=max(1.0, t_end - time.time()))
    alive = [p.pid for p in procs if p.is_alive()]
    for p in procs:
        if p.is_alive():
            p.kill()
    res = sorted(q.get(timeout=5) for _ in procs) if not alive and all(p.exitcode == 0 for p in procs) else []
    ok = bool(res) and all(b == 0 and gb == 0 and e == 0 for _, b, gb, e, _ in res)
    print(json.dumps({"world": a.world, "calls": a.calls, "ok": ok, "killed": alive,
                      "ranks": [{"rank": r, "mismatches": b, "graph_mismatch": gb, "err": e, "us_per_call": round(t, 2)}
                                for r, b, gb, e, t in res],
                      "exitcodes": [p.exitcode for p in procs]}), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
