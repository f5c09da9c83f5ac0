"""Multi-process CPU reference CG over torch.distributed (gloo).

Runs the reference recurrence (CUDACG.cu:244-352) with the SAME partition and
halo plan the GPU solver uses (native ``make_layout``), each process owning its
rows, exchanging halo ranges with isend/irecv and all-reducing the two dot
products.  It is the CPU rehearsal of the distributed path (world_size > 1 without
a GPU) and an oracle for the RCCL solver.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import native
from .plan import layout as _layout


def _allreduce(v: float) -> float:
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t)
    return float(t.item())


def cpu_cg_distributed(spec, maxit: int = 2000, tol: float = 1e-7, group=None) -> Dict:
    """Solve on the current gloo process group; returns this rank's x plus global stats."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    ns = spec.native() if hasattr(spec, "native") else spec
    L = _layout(ns, world, rank)
    rowptr, cols, vals = native().host_csr(ns, world, rank)
    n = L.n_local
    b = native().host_rhs(ns, L.row_begin, L.row_end)
    x = np.zeros(n)
    r = b.copy()
    p = np.zeros(L.ext_len)
    own = slice(L.own_off, L.own_off + n)
    p[own] = b
    # per-row segment ids for a vectorised CSR SpMV
    row_of = np.repeat(np.arange(n), np.diff(rowptr))

    def spmv(v_ext: np.ndarray) -> np.ndarray:
        return np.bincount(row_of, weights=vals * v_ext[cols], minlength=n)

    def halo(v_ext: np.ndarray) -> None:
        if world == 1:
            return
        if L.allgather:  # the RCCL path's ncclAllGather of equal blocks, on gloo
            blk = torch.from_numpy(np.ascontiguousarray(v_ext[L.own_off:L.own_off + L.block]))
            parts = [torch.empty(L.block, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(parts, blk, group=group)
            for q, t in enumerate(parts):
                v_ext[q * L.block:(q + 1) * L.block] = t.numpy()
            return
        reqs = []
        bufs = []
        for peer, g0, cnt in L.sends:
            i0 = L.ext_index(g0)
            t = torch.from_numpy(np.ascontiguousarray(v_ext[i0:i0 + cnt]))
            bufs.append(t)
            reqs.append(dist.isend(t, peer, group=group))
        recv_bufs = []
        for peer, g0, cnt in L.recvs:
            t = torch.empty(cnt, dtype=torch.float64)
            recv_bufs.append((L.ext_index(g0), cnt, t))
            reqs.append(dist.irecv(t, peer, group=group))
        for q in reqs:
            q.wait()
        for i0, cnt, t in recv_bufs:
            v_ext[i0:i0 + cnt] = t.numpy()

    rho = math.sqrt(_allreduce(float(r @ r)) if world > 1 else float(r @ r))
    rho = rho * rho
    hist = []
    it = 0
    converged = False
    breakdown = False
    while it < maxit:
        halo(p)
        Ap = spmv(p)
        tmp = float(p[own] @ Ap)
        tmp = _allreduce(tmp) if world > 1 else tmp
        alpha = rho / tmp
        x += alpha * p[own]
        r += -alpha * Ap
        it += 1
        rhop = rho
        rr = float(r @ r)
        rho = math.sqrt(_allreduce(rr) if world > 1 else rr)
        hist.append(rho)
        if not math.isfinite(rho):
            breakdown = True
            break
        if rho < tol:
            converged = True
            break
        rho = rho * rho
        beta = rho / rhop
        p[own] = beta * p[own] + r
    return {
        "x": x,
        "row_begin": L.row_begin,
        "iterations": it,
        "converged": converged,
        "breakdown": breakdown,
        "rnorm": hist[-1] if hist else float("nan"),
        "rnorm_history": np.array(hist),
    }


def gather_x(local: Dict, n_global: Optional[int] = None) -> np.ndarray:
    """All-gather the distributed solution (gloo) into a full vector on every rank."""
    world = dist.get_world_size()
    parts = [None] * world
    dist.all_gather_object(parts, (local["row_begin"], local["x"]))
    parts.sort(key=lambda t: t[0])
    return np.concatenate([p[1] for p in parts])
