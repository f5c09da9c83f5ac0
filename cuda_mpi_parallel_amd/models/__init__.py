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
``randspd``    banded, irregular, strictly diag. dominant   BASELINE.json config 5
=============  ===========================================  ==========================
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .. import native

PROBLEMS = ("demo", "poisson2d", "poisson3d", "randspd")


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

    def native(self):
        return native().ProblemSpec(self.problem, self.n, self.rows, self.band, self.density, self.seed, self.rhs)

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


def make_problem(name: str = "demo", **kw) -> ProblemSpec:
    """``make_problem("poisson2d", n=4096)``; non-demo problems default to a random RHS
    (BASELINE.json:5 "random RHS"); randspd defaults to rows=100000, band=64."""
    name = {"random-spd": "randspd", "random": "randspd"}.get(name, name)
    if name not in PROBLEMS:
        raise ValueError(f"unknown problem {name!r}; choose from {PROBLEMS}")
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


__all__ = ["PROBLEMS", "ProblemSpec", "make_problem", "host_csr", "to_scipy", "rhs"]
