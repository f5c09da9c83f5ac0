"""High-level CG drivers.

``CGSolver`` wraps the native distributed GPU solver (``csrc/gpu/solver.cpp``):
on-device generation of this rank's rows, fused HIP kernels, device-resident
scalars, RCCL all-reduce + halo on side streams, hipGraph-captured iteration
pairs.  ``device="cpu"`` runs the CPU reference path instead (single process,
``sim_ranks`` virtual ranks, or — under torch.distributed/gloo — one process
per rank).

Semantics follow the reference (CUDACG.cu:235-352): x0 = 0, r0 = p0 = b,
stop when ||r||_2 < tol (absolute) after the x/r update, at most ``maxit``
iterations, no abort on non-positive curvature.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .. import native
from ..models import ProblemSpec, make_problem
from ..parallel import dist as _dist


def _opts(maxit=2000, tol=1e-7, **kw):
    """Native CgOptions; keyword names as in csrc/include/mcg/cg.hpp (format, blocks_per_cu,
    spmv_variant, recurrence, ...)."""
    ctor = {"check_every", "overlap", "use_graph", "force_comm", "format", "blocks_per_cu", "spmv_variant",
            "recurrence"}
    o = native().CgOptions(maxit=maxit, tol=tol, **{k: v for k, v in kw.items() if k in ctor})
    for k, v in kw.items():
        if k not in ctor:
            if not hasattr(o, k):
                raise TypeError(f"unknown solver option {k!r}")
            setattr(o, k, v)
    return o


class CGSolver:
    """Distributed GPU CG for one rank (one process per GPU, or a single GPU).

    ``format="auto"`` (default) picks what both CLIs pick: the reference's CSR and two-reduction
    order for the built-in demo, SELL-64/c8 (falling back to /dia4, /diav, /d16, tiles as the matrix
    allows) with the auto recurrence (single-reduction pass) for every other problem, so
    ``solve("poisson2d")`` runs the Ap-recomputing line carry."""

    def __init__(self, spec: ProblemSpec, maxit: int = 2000, tol: float = 1e-7, check_every: int = 32,
                 overlap: bool = True, use_graph: bool = True, format: str = "auto", force_comm: bool = False,
                 blocks_per_cu: int = 0, env: Optional[_dist.DistEnv] = None, comm=None, comm_mode: str = "single",
                 halo_transport: str = "auto", allreduce: str = "auto", rehearse_ranks: bool = False, **tuning):
        """``halo_transport`` / ``allreduce`` (P > 1, a communicator built here): "auto" maps the
        neighbours' halo buffers (the lean carries' in-kernel halo) and every rank's IPC all-reduce
        mailbox next to RCCL, and the solver's transport probe keeps the fastest correct pair at the
        first reset; "rccl" keeps RCCL only; ``allreduce="ipc"`` forces the mailboxes.
        ``rehearse_ranks``: the P processes share GPU 0 (collectives: IPC mailboxes and copy engines,
        no RCCL) -- the real P-rank recurrence on one GPU, as ``bench.py --rehearse-ranks --allreduce ipc``."""
        if format == "auto":
            demo = getattr(spec, "problem", "") == "demo"
            format = "csr" if demo else "sellc8"
            if not demo:
                tuning.setdefault("recurrence", -1)
        if halo_transport not in ("auto", "rccl") or allreduce not in ("auto", "rccl", "ipc"):
            raise ValueError(f"halo_transport auto|rccl, allreduce auto|rccl|ipc; got {halo_transport!r}, {allreduce!r}")
        self.spec = spec
        self.env = env or _dist.dist_env()
        rehearse = rehearse_ranks and self.env.world > 1
        if rehearse:
            import torch

            torch.cuda.set_device(0)
        else:
            _dist.set_device(self.env)
        peer = False
        if comm is None and (self.env.world > 1 or force_comm):
            _dist.init_process_group(self.env)
            if rehearse:  # every rank on GPU 0: the IPC all-reduce and the copy-engine halo (RCCL refuses)
                comm = _dist.peer_halo(native().NullComm(self.env.rank, self.env.world), self.env, ipc_allreduce=True)
                peer = True
            else:
                comm = _dist.bootstrap_comm(self.env, force=force_comm, mode=comm_mode)
                if self.env.world > 1 and halo_transport == "auto":
                    probe_ar = allreduce == "auto"
                    comm = _dist.peer_halo(comm, self.env, ipc_allreduce=probe_ar or allreduce == "ipc",
                                           halo_via_inner=True, tolerant=probe_ar)
                    if probe_ar:
                        comm.ipc_allreduce = False  # the transport probe decides
                    peer = True
        self.comm = comm
        if halo_transport == "rccl":
            tuning.setdefault("halo_pull", 0)  # no mapped peers: every ghost line exchanged
        self.opts = _opts(maxit, tol, check_every=check_every, overlap=overlap, use_graph=use_graph,
                          force_comm=force_comm, format=format, blocks_per_cu=blocks_per_cu, **tuning)
        self._s = native().Solver(spec.native(), self.opts, self.env.rank, self.env.world, comm)
        self._s.setup()
        if peer:  # map the peers' registered halo buffers (collective; the first reset checks the mapping)
            _dist.attach_peer_halo(comm, self.env, tolerant=not rehearse)

    # --- solve to tolerance (reference semantics) ---
    def solve(self, resume: bool = False) -> Dict:
        """Solve to tol / maxit.  ``resume=True`` continues from the state loaded by
        :meth:`load_checkpoint` instead of restarting from x0 = 0."""
        res = self._s.solve(resume)
        res["x_local"] = self._s.x_local()
        res["row_begin"] = self._s.layout["row_begin"]
        return res

    # --- fixed-work benchmark mode ---
    def reset(self) -> None:
        self._s.reset()

    def run(self, iterations: int) -> None:
        """Enqueue `iterations` more CG iterations (asynchronous)."""
        self._s.run_iterations(int(iterations))

    def synchronize(self) -> None:
        self._s.synchronize()

    def finalize(self) -> None:
        self._s.finalize()

    def result(self) -> Dict:
        return self._s.result()

    def x_local(self) -> np.ndarray:
        return self._s.x_local()

    def true_residual_norm(self) -> float:
        return self._s.true_residual_norm()

    # --- checkpoint / resume (per-rank files "<prefix>.rank<r>") ---
    def save_checkpoint(self, prefix: str) -> None:
        self._s.save_checkpoint(prefix)

    def load_checkpoint(self, prefix: str) -> None:
        self._s.load_checkpoint(prefix)

    @property
    def info(self) -> Dict:
        return self._s.info

    @property
    def layout(self) -> Dict:
        return self._s.layout


def solve(problem: str = "demo", device: str = "gpu", sim_ranks: int = 1, maxit: int = 2000, tol: float = 1e-7,
          **kw) -> Dict:
    """One-call solve.  ``solve()`` with no arguments is the reference's demo."""
    spec_kw = {k: kw.pop(k) for k in ("n", "rows", "band", "density", "seed", "rhs", "spread", "scramble", "coef",
                                      "nnz_per_row", "matrix", "b", "reorder") if k in kw}
    if "matrix" in spec_kw:  # solve(matrix=A_or_path, b=...): a user matrix (kind csr)
        problem = "csr"
    spec = make_problem(problem, **spec_kw)
    perm = getattr(spec, "perm", None)  # reordered user matrix: hand x back in the caller's numbering
    if device == "cpu":
        o = _opts(maxit, tol)
        C = native()
        r = C.cpu_cg_partitioned(spec.native(), sim_ranks, o) if sim_ranks > 1 else C.cpu_cg(spec.native(), o)
        if perm is not None:
            r["x"] = spec.unpermute(r["x"])
        return r
    s = CGSolver(spec, maxit=maxit, tol=tol, **kw)
    r = s.solve()
    if perm is not None and s.env.world == 1:
        r["x_local"] = spec.unpermute(r["x_local"])
    return r


__all__ = ["CGSolver", "solve"]
