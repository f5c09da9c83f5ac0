"""Process-group bootstrap: one process per GPU under torchrun, RCCL for the solver.

``torch.distributed`` (gloo, host side) is used only for rendezvous, barriers and
shipping the two ``ncclUniqueId``s; the solver's own collectives are native RCCL
calls issued from C++ on the solver's HIP streams (``csrc/gpu/comm.cpp``), so no
Python is on the per-iteration path.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .. import native


@dataclass(frozen=True)
class DistEnv:
    rank: int
    world: int
    local_rank: int

    @property
    def is_distributed(self) -> bool:
        return self.world > 1


def dist_env() -> DistEnv:
    """RANK / WORLD_SIZE / LOCAL_RANK from the torchrun environment (defaults: single rank)."""
    return DistEnv(
        rank=int(os.environ.get("RANK", "0")),
        world=int(os.environ.get("WORLD_SIZE", "1")),
        local_rank=int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))),
    )


def init_process_group(env: DistEnv, backend: str = "gloo") -> None:
    """Initialise torch.distributed if running multi-rank (MASTER_ADDR/PORT from torchrun)."""
    if env.world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=env.rank, world_size=env.world)


def bootstrap_comm(env: DistEnv, force: bool = False, mode: str = "single"):
    """Create the native RCCL communicator(s) for this rank (None for a single rank unless
    ``force``).  Rank 0 draws the unique ids and broadcasts them over the torch.distributed
    store-backed process group.  ``mode``: "dual" = a reduce and a halo communicator (halo on the
    side stream, overlapped); "single" = one communicator, every collective in one stream order."""
    if env.world == 1 and not force:
        return None
    if mode not in ("dual", "single"):
        raise ValueError(f"comm mode must be dual or single, got {mode!r}")
    C = native()
    nids = 2 if mode == "dual" else 1
    if env.world == 1:
        ids = [C.unique_id() for _ in range(nids)]
    else:
        if not dist.is_initialized():
            raise RuntimeError("bootstrap_comm needs torch.distributed initialised (call init_process_group)")
        ids = [C.unique_id() for _ in range(nids)] if env.rank == 0 else [None] * nids
        dist.broadcast_object_list(ids, src=0)
    return C.Comm(env.rank, env.world, *ids)


def peer_halo(inner, env: DistEnv, ipc_allreduce: bool = False, halo_via_inner: bool = False,
              tolerant: bool = False):
    """Wrap a communicator so that the halo moves without RCCL (native ``PeerHaloComm``: the
    neighbours' buffers mapped through IPC handles -- pulled by copy engines, or read by the lean
    passes themselves, PassForm::halo_pull); the all-reduce stays on ``inner`` unless
    ``ipc_allreduce``: then every rank's mailbox is mapped here (collective) and the all-reduce runs
    through them (ipc_allreduce.hip) -- real P-rank sums with no RCCL, e.g. P processes on one GPU.
    ``halo_via_inner``: only the mapping (the lean passes' in-kernel halo); every halo exchange that
    remains goes to ``inner`` (RCCL's send/recv).  Call :func:`attach_peer_halo` after the solver's
    ``setup()``.  ``tolerant``: a rank that cannot allocate, export or map the mailboxes leaves them
    unmapped instead of raising (every rank then skips them: the solver's transport probe agrees on it,
    and the all-reduce stays on ``inner``)."""
    import sys

    comm = native().PeerHaloComm(inner, env.rank, env.world)
    comm.halo_via_inner = halo_via_inner
    if ipc_allreduce:
        try:
            mine = comm.mailbox_handle()
        except Exception as e:  # noqa: BLE001
            if not tolerant:
                raise
            print(f"[mcg] rank {env.rank}: IPC all-reduce mailbox unavailable ({e})", file=sys.stderr, flush=True)
            mine = b""
        allb = [mine]
        if env.world > 1:
            if not dist.is_initialized():
                raise RuntimeError("peer_halo(ipc_allreduce=True) needs torch.distributed initialised")
            allb = [None] * env.world
            dist.all_gather_object(allb, mine)
        if all(allb):
            try:
                comm.attach_mailbox(allb)
            except Exception as e:  # noqa: BLE001
                if not tolerant:
                    raise
                print(f"[mcg] rank {env.rank}: IPC all-reduce mailboxes not mapped ({e})", file=sys.stderr, flush=True)
        elif not tolerant:
            raise RuntimeError("a rank could not export its IPC all-reduce mailbox")
    return comm


def attach_peer_halo(comm, env: DistEnv, tolerant: bool = False) -> bool:
    """Exchange every rank's IPC handles (registered by the solver's setup) over torch.distributed
    and map the peers' halo buffers.  Collective: every rank calls it once, after ``setup()``.
    ``tolerant``: a rank whose mapping fails stays unattached instead of raising (the solver then
    agrees with every rank, at its next reset, not to read peer rows: the in-kernel halo's check);
    returns whether this rank attached."""
    import sys

    mine = comm.local_handles()
    if env.world == 1:
        allb = [mine]
    else:
        if not dist.is_initialized():
            raise RuntimeError("attach_peer_halo needs torch.distributed initialised")
        allb = [None] * env.world
        dist.all_gather_object(allb, mine)
    try:
        comm.attach(allb)
    except Exception as e:  # noqa: BLE001
        if not tolerant:
            raise
        print(f"[mcg] rank {env.rank}: peer mapping failed ({e}); the halo stays on the inner communicator",
              file=sys.stderr, flush=True)
        return False
    return True


def set_device(env: DistEnv) -> int:
    """Bind this process to its GPU (LOCAL_RANK) — like the reference's cudaSetDevice(0)."""
    n = torch.cuda.device_count()
    if n == 0:
        raise RuntimeError("Device Set failed")  # CUDACG.cu:88-91 wording; no HIP device visible
    dev = env.local_rank % n
    torch.cuda.set_device(dev)
    return dev
