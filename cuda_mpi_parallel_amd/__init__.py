"""cuda_mpi_parallel_amd — MI355X-native distributed conjugate-gradient framework.

A from-scratch re-design of the capabilities of ``Yan12345678/CUDA-MPI-parallel``
(reference: a single-file cuBLAS/cuSPARSE fp64 CG solver, ``CUDACG.cu``) for AMD
Instinct MI355X (gfx950 / CDNA4):

* native C++17 runtime + hand-written HIP kernels (``csrc/``) compiled for gfx950:
  fused CSR / SELL-64 SpMV, fused residual update, fixed-order reductions,
  on-device problem generators;
* 1-D row partition across GPUs, boundary-row halo exchange and the per-iteration
  dot-product all-reduces on RCCL over xGMI (one process or one thread per GPU);
* a CPU reference path (single process, virtual ranks, and multi-process gloo).

Package layout::

    models/    problem families (demo 3x3, 2-D/3-D Poisson, random SPD)
    ops/       torch-tensor wrappers over the hand-written kernels
    parallel/  partition / halo plans, RCCL bootstrap over torch.distributed,
               multi-process CPU reference (gloo)
    solver/    high-level CG drivers (GPU native solver, CPU reference)
    utils/     output helpers (reference x format, JSON result lines)

``torch`` is imported before the native extension on purpose: torch ships its own
``libamdhip64.so.7`` / ``librccl.so.1``; loading it first makes the extension bind
to the same HIP runtime and RCCL (matching SONAMEs) instead of a second copy.
"""
from __future__ import annotations

import importlib as _importlib
import os as _os

import torch as _torch  # noqa: F401  (must precede the native extension; see docstring)

_C = None  # the native extension, loaded on first use by native()
_IMPORT_ERROR = None

__version__ = "0.2.0"


def native():
    """Return the native extension module, raising loudly if it was not built.

    Loaded lazily so that launchers (``parallel/launch.py``) can start the per-GPU ranks
    before this process maps any HIP code."""
    global _C, _IMPORT_ERROR
    if _C is None:
        try:
            mod = _importlib.import_module(__name__ + "._C")
        except ImportError as e:
            _IMPORT_ERROR = e
            raise ImportError(
                "cuda_mpi_parallel_amd native extension (_C) is not built: run `make -j8` "
                "or `python -c 'import __graft_entry__ as g; g.build()'` in the repo root "
                f"({_IMPORT_ERROR})"
            ) from e
        _C = mod
    return _C


def repo_root() -> str:
    return _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))


def cli_path() -> str:
    """Path of the native ``mcg-cg`` CLI binary."""
    return _os.path.join(repo_root(), "bin", "mcg-cg")


from . import models, ops, parallel, solver, utils  # noqa: E402,F401
from .models import CsrProblem, ProblemSpec, csr_problem, make_problem  # noqa: E402,F401
from .solver import CGSolver, solve  # noqa: E402,F401
