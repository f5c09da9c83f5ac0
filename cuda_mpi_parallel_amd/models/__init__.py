"""Problem families — the "models" this framework solves.

Each family is defined row-by-row by a pure function of the global row index in
``csrc/include/mcg/problem.hpp`` (shared by the host reference path and the
on-device generators), so a rank generates only its owned rows and the RHS is
independent of the number of ranks.

=============  ===========================================  ==========================
name           matrix                                       reference / config
=============  ===========================================  ==========================
``demo``       the reference's 3x3 indefinite system        CUDACG.cu:74-117,136-141
``poisson2d``  5-pt Dirichlet Laplacian, n = N^2            BASELINE.json configs 1-3
``poisson3d``  7-pt Dirichlet Laplacian, n = N^3            BASELINE.json config 4
               (both: ``coef=1`` = heterogeneous diffusion,  CUDACG.cu:93-117 (arbitrary
               a seeded random conductivity field)           stencil values)
``randspd``    banded / wide (spread) multi-diagonal, or    BASELINE.json config 5
               scrambled (P^T A P, irregular); strictly
               diagonally dominant
``csr``        a user matrix: SciPy / NumPy CSR arrays or a  CUDACG.cu:93-117,213-216
               Matrix Market file (:func:`csr_problem`)       (the reference's input)
=============  ===========================================  ==========================
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .. import native

PROBLEMS = ("demo", "poisson2d", "poisson3d", "randspd", "csr")


@dataclass(frozen=True)
class ProblemSpec:
    """Python-side description of a problem; ``.native()`` builds the C++ spec."""

    problem: str = "demo"
    n: int = 3            # grid edge N (poisson2d: N^2 rows, poisson3d: N^3 rows)
    rows: int = 0         # randspd rows
    band: int = 0         # randspd half bandwidth
    density: float = 0.5  # randspd mean pair density
    seed: int = 1234
    rhs: str = "reference"  # reference | random | ones
    spread: int = 0       # randspd: > 0 = the band candidate offsets drawn over [1, spread] ("wide")
    scramble: int = 0     # randspd: 1 = P^T A P with a seeded random permutation P (genuinely irregular)
    coef: int = 0         # poisson2d/3d: 1 = variable coefficients (random conductivity field, symmetric)

    def native(self):
        return native().ProblemSpec(self.problem, self.n, self.rows, self.band, self.density, self.seed, self.rhs,
                                    self.spread, self.scramble, self.coef)

    @property
    def n_rows(self) -> int:
        return int(self.native().n_rows)

    @property
    def nnz(self) -> Optional[int]:
        v = int(self.native().closed_form_nnz)
        return None if v < 0 else v

    def footprint_bytes(self, ranks: int = 1, idx64: bool = False) -> int:
        """Approximate device bytes per rank: CSR + 3 ext vectors + 3 owned vectors."""
        n = self.n_rows
        nnz = self.nnz if self.nnz is not None else n * (1 + 2 * self.band * self.density)
        per_rank_rows = n / ranks
        return int(nnz / ranks * 12 + per_rank_rows * ((8 if idx64 else 4) + 6 * 8))


class CsrProblem:
    """A user matrix (kind ``csr``): the same interface as :class:`ProblemSpec`.

    The native ``HostMatrix`` owns the arrays; every rank reads the whole matrix on the host and
    uploads only its own rows (partition and ghost plan from the actual columns).  ``rhs``:
    ``"reference"`` = the given ``b`` (ones when none is given), ``"ones"``, ``"random"``.
    ``reorder="rcm"`` applies a reverse Cuthill-McKee permutation (SciPy) first, which turns
    most mesh matrices into banded ones (column-window halos instead of the all-gather);
    :meth:`unpermute` maps a solution back to the original numbering.
    """

    problem = "csr"

    def __init__(self, matrix, rhs: str = "reference", seed: int = 1234, perm: Optional[np.ndarray] = None):
        self.matrix = matrix
        self.rhs = rhs
        self.seed = seed
        self.perm = perm
        self._spec = matrix.spec(rhs, seed)

    def native(self):
        return self._spec

    @property
    def n_rows(self) -> int:
        return int(self.matrix.n)

    @property
    def nnz(self) -> int:
        return int(self.matrix.nnz)

    def unpermute(self, x: np.ndarray) -> np.ndarray:
        """Solution of the permuted system -> original row order."""
        if self.perm is None:
            return np.asarray(x)
        out = np.empty_like(np.asarray(x))
        out[self.perm] = x
        return out


def csr_problem(a, b=None, rhs: str = "reference", seed: int = 1234, reorder: Optional[str] = None) -> CsrProblem:
    """A :class:`CsrProblem` from a SciPy sparse matrix, an ``(indptr, indices, data)`` triple or
    a Matrix Market path (``.mtx``)."""
    perm = None
    if isinstance(a, str):
        if reorder is None and b is None:
            return CsrProblem(native().HostMatrix.read_mtx(a), rhs, seed)
        import scipy.io

        a = scipy.io.mmread(a)
    if isinstance(a, tuple):
        indptr, indices, data = a
    else:
        import scipy.sparse as sp

        m = sp.csr_matrix(a)
        if m.shape[0] != m.shape[1]:
            raise ValueError("matrix must be square")
        if reorder == "rcm":
            from scipy.sparse.csgraph import reverse_cuthill_mckee

            perm = np.asarray(reverse_cuthill_mckee(m, symmetric_mode=True), dtype=np.int64)
            m = m[perm][:, perm].tocsr()
            if b is not None:
                b = np.asarray(b, dtype=np.float64)[perm]
        elif reorder is not None:
            raise ValueError(f"unknown reorder {reorder!r}")
        m.sort_indices()
        indptr, indices, data = m.indptr, m.indices, m.data
    H = native().HostMatrix(np.asarray(indptr, dtype=np.int64), np.asarray(indices, dtype=np.int64),
                            np.asarray(data, dtype=np.float64), None if b is None else np.asarray(b, np.float64))
    return CsrProblem(H, rhs, seed, perm)


def make_problem(name: str = "demo", **kw):
    """``make_problem("poisson2d", n=4096)``; non-demo problems default to a random RHS
    (BASELINE.json:5 "random RHS"); randspd defaults to rows=100000, band=64;
    ``make_problem("csr", matrix=A_or_path, b=None)`` wraps a user matrix."""
    name = {"random-spd": "randspd", "random": "randspd", "mtx": "csr"}.get(name, name)
    if name not in PROBLEMS:
        raise ValueError(f"unknown problem {name!r}; choose from {PROBLEMS}")
    if name == "csr":
        return csr_problem(kw.pop("matrix"), **kw)
    if name != "demo":
        kw.setdefault("rhs", "random")
    if name == "randspd":
        kw.setdefault("rows", 100000)
        kw.setdefault("band", 64)
        m = kw.pop("nnz_per_row", None)  # mean nonzeros per row -> candidate-pair density
        if m is not None:
            kw["density"] = min(1.0, max(0.0, (float(m) - 1.0) / (2.0 * kw["band"])))
    if name in ("poisson2d", "poisson3d"):
        kw.setdefault("n", 1024 if name == "poisson2d" else 128)
    return ProblemSpec(problem=name, **kw)


def host_csr(spec: ProblemSpec, world: int = 1, rank: int = 0):
    """(rowptr int64, cols int32 in ext coords, vals f64) of rank's owned rows (host build)."""
    return native().host_csr(spec.native(), world, rank)


def to_scipy(spec: ProblemSpec):
    """Global matrix as scipy.sparse.csr_matrix (tests / oracles; small sizes only)."""
    import scipy.sparse as sp

    rowptr, cols, vals = host_csr(spec)
    n = spec.n_rows
    return sp.csr_matrix((vals, cols.astype(np.int64), rowptr), shape=(n, n))


def rhs(spec: ProblemSpec, r0: int = 0, r1: Optional[int] = None) -> np.ndarray:
    r1 = spec.n_rows if r1 is None else r1
    return native().host_rhs(spec.native(), r0, r1)


__all__ = ["PROBLEMS", "ProblemSpec", "CsrProblem", "csr_problem", "make_problem", "host_csr", "to_scipy", "rhs"]
