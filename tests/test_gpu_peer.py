"""The copy-engine halo transport (PeerHaloComm, csrc/gpu/peer_halo.cpp) across PROCESSES on one GPU:
IPC-mapped peer buffers, hipMemcpyDeviceToDeviceNoCU pulls, stream write / wait-value flags.  The
reference has no communication at all (CUDACG.cu:87, one device); this is the north star's halo and
all-gather moved off the compute units."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


def _port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


@pytest.mark.parametrize("world,problem", [(2, "poisson2d"), (4, "scrambled")])
def test_peer_halo_processes_pull_the_owners_rows(world, problem):
    """P processes on device 0 exchange rank-tagged rows over the copy engines, several rounds with new
    values each: every ghost row equals its owner's row -- the 2-D window halo (neighbour lines) and
    the all-gather layout of the scrambled family (every peer's block, one copy stream per peer)."""
    p = _run([sys.executable, "-u", "bench/peer_halo_check.py", "--world", str(world), "--problem", problem,
              "--rounds", "4", "--port", str(_port())])
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["ok"] and all(r["mismatches"] == 0 for r in line["ranks"])
    assert all(r["allgather"] == (problem == "scrambled") for r in line["ranks"])
    assert all(r["recv_ranges"] >= (world - 1 if problem == "scrambled" else 1) for r in line["ranks"])


def test_bench_sdma_halo_rehearsal_on_one_gpu():
    """bench.py at P = 2 under torchrun on one GPU with the copy-engine halo (--halo-transport sdma):
    the solver's halo goes through PeerHaloComm inside the 32-iteration graphs (flags replayed),
    collectives of the all-reduce move nothing (rehearsal); every rank ok and latched together."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--rehearse-ranks", "--grid",
           "2048", "--steps", "64", "--warmup", "8", "--phases", "0", "--watchdog", "60", "--halo-transport", "sdma"]
    p = _run(cmd)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["check"]["ok"] and line["n_gpus"] == 2
    # the lean 2-D carry (runs of >= 3 lines: 2048^2 at P = 2) reads its ghost lines in-kernel from the
    # mapped neighbour (halo_pull auto)
    assert line["config"]["halo_transport"].startswith("in-kernel") and line["check"]["lean_only"]


@pytest.mark.parametrize("world,problem,n,pull,coef", [(2, "poisson2d", 2048, -1, 0), (4, "poisson2d", 2048, -1, 0),
                                                       (2, "poisson2d", 2048, 0, 0), (4, "poisson3d", 128, -1, 0),
                                                       (2, "poisson2d", 1024, -1, 1)])
def test_ipc_ranks_real_recurrence_matches_one_rank(world, problem, n, pull, coef):
    """P processes on ONE GPU run the real P-rank recurrence -- the IPC all-reduce
    (mailboxes mapped through IPC handles, rank-order sums) and the peer-mapped halo (the in-kernel
    halo, or the copy-engine pulls with halo_pull 0), captured in 32-iteration graphs -- and agree with
    one rank to <= 1e-13 over 40 iterations."""
    p = _run([sys.executable, "-u", "bench/ipc_ranks.py", "--world", str(world), "--problem", problem, "--n", str(n),
              "--halo-pull", str(pull), "--coef", str(coef), "--iters", "40", "--port", str(_port())], timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["ok"], line
    # graphs hold the pulled iterations; the copy-engine exchanges run eager (they replay without their
    # order from a graph: PeerHaloComm::halo_capturable)
    assert all(r["halo_pull"] == (pull != 0) and r["graphs"] == (pull != 0) and r["graph_fallbacks"] == 0
               for r in line["ranks"]), line
    assert line["gap_rnorm"] <= 1e-13 and line["true_gap"] <= 1e-8, line


@pytest.mark.parametrize("world,problem,n,pick", [(2, "poisson2d", 2048, 0), (2, "poisson2d", 2048, 1),
                                                  (2, "poisson3d", 128, 0), (2, "poisson2d", 2048, -1),
                                                  (8, "poisson2d", 4096, -1)])
def test_ipc_ranks_transport_probe_arms(world, problem, n, pick):
    """the transport probe at the first reset of a real 2-process solve on one GPU (IPC
    all-reduce, peer-mapped buffers) runs the pulled and the exchanged arm, finds the pulled one bit for
    bit the exchanged one, and keeps what it is told (or the faster: -1) on both ranks alike; the kept
    transport then runs the solve, which matches one rank -- the choice is numerically neutral."""
    p = _run([sys.executable, "-u", "bench/ipc_ranks.py", "--world", str(world), "--problem", problem, "--n", str(n),
              "--probe-pick", str(pick), "--iters", "40", "--port", str(_port())], timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["ok"] and line["gap_rnorm"] <= 1e-13, line
    rk = line["ranks"]
    assert all(r["probe_ran"] and r["probe_pull_bitwise"] and r["probe_pull_us"] > 0 and r["probe_xchg_us"] > 0
               for r in rk), rk
    assert len({r["halo_pull"] for r in rk}) == 1 and (pick < 0 or rk[0]["halo_pull"] == bool(pick)), rk
    # the arms' times are the mean over the ranks: the same numbers on every rank
    assert len({(r["probe_pull_us"], r["probe_xchg_us"]) for r in rk}) == 1, rk


@pytest.mark.parametrize("problem,recurrence,pipe_rr", [("poisson2d", 2, 0), ("poisson2d", 2, 10), ("scrambled", 1, 0)])
def test_ipc_ranks_single_buffer_exchanges(problem, recurrence, pipe_rr):
    """the copy-engine halo on buffers that are NOT parity-alternating -- the pipelined pass's w
    (rewritten by the update right after its exchange; with residual replacement also r, p, s) and the
    split pass's p on the all-gather layout -- across processes, with the IPC all-reduce: the owner's
    stream waits for its readers' done flags before rewriting (Communicator::halo_fence), so the
    2-process solve matches one rank."""
    p = _run([sys.executable, "-u", "bench/ipc_ranks.py", "--world", "2", "--problem", problem, "--n", "512",
              "--recurrence", str(recurrence), "--pipe-rr", str(pipe_rr), "--iters", "60", "--tol", "1e-11",
              "--port", str(_port())], timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["ok"] and not any(r["halo_pull"] for r in line["ranks"]), line


def test_bench_ipc_allreduce_rehearsal_is_a_real_solve():
    """bench.py --rehearse-ranks --allreduce ipc: the P-rank bench on one GPU with the IPC all-reduce is a
    real solve, so its check requires the recurrence residual to track ||b - A x||."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--rehearse-ranks", "--grid",
           "2048", "--steps", "64", "--warmup", "8", "--phases", "0", "--watchdog", "60", "--allreduce", "ipc"]
    p = _run(cmd)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["check"]["ok"] and line["check"]["true_gap_rel"] <= 1e-8, line["check"]
    assert line["config"]["allreduce"].startswith("ipc") and "real" in line["metric"]
