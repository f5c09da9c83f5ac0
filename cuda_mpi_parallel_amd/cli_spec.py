"""The one flag table of both command-line entry points.

``bin/mcg-cg`` (csrc/cli/main.cpp, hand-rolled parser, one host thread per GPU) and
``python -m cuda_mpi_parallel_amd`` (argparse built from this table, one process per GPU through
parallel/launch.py) accept exactly these flags with the same spellings and value forms;
tests/test_cli_parity.py runs every entry through both.  With no flags both behave like the
reference binary (CUDACG.cu:41-366): the built-in 3x3 system, ``%f`` per line, ``Success``.

Each entry: (flag, example value or None for a switch, help).
"""
from __future__ import annotations

TRI = "auto|on|off"

FLAGS = [
    # problem
    ("--problem", "demo", "demo | poisson2d | poisson3d | randspd | csr"),
    ("--n", "16", "grid edge N (poisson2d: N^2 rows, poisson3d: N^3)"),
    ("--rows", "2000", "randspd: global rows"),
    ("--band", "8", "randspd: candidate offsets per side (half bandwidth when --spread 0)"),
    ("--density", "0.3", "randspd: mean candidate-pair density"),
    ("--nnz-per-row", "5", "randspd: mean nonzeros per row (sets --density)"),
    ("--spread", "0", "randspd: > 0 = candidate offsets drawn over [1, spread] (wide multi-diagonal)"),
    ("--scramble", "0", "randspd: 1 = P^T A P with a seeded random permutation (genuinely irregular rows)"),
    ("--coef", "0", "poisson2d/3d: 1 = variable coefficients (seeded random conductivity field)"),
    ("--matrix", None, "FILE.mtx: a user matrix (problem csr), Matrix Market coordinate"),
    ("--rhs-file", None, "FILE: right-hand side of --matrix (Matrix Market array or one value per line)"),
    ("--rhs", "reference", "reference | random | ones"),
    ("--seed", "1234", "matrix / rhs seed"),
    # where
    ("--device", "cpu", "gpu | cpu"),
    ("--gpus", "1", "P ranks, one GPU each"),
    ("--sim-ranks", "1", "cpu: P virtual ranks in one process"),
    # stopping (CUDACG.cu:244-245)
    ("--maxit", "2000", "iteration limit"),
    ("--tol", "1e-7", "absolute ||r||_2 tolerance"),
    ("--rtol", "0", "> 0: stop on ||r|| < rtol ||b|| instead"),
    ("--check-every", "32", "host polls the device latch every K iterations"),
    ("--fixed-iters", "0", "> 0: benchmark mode, exactly K iterations (tol off)"),
    ("--warmup", "0", "benchmark mode: untimed iterations first"),
    ("--watchdog", "0", "> 0: fail (and abort RCCL) when a poll interval makes no progress for S seconds"),
    # solver form / kernels
    ("--format", "csr", "csr | sell | sell16 | sellc8"),
    ("--recurrence", "auto", "auto | two | single | pipelined"),
    ("--pipe-rr", "0", "pipelined CG: residual replacement every K iterations (0 = off)"),
    ("--interleave", "auto", TRI + ": {r, Ap} 16-B pairs (single-reduction SELL)"),
    ("--window", "auto", TRI + ": LDS column windows (long banded rows)"),
    ("--carry", "auto", TRI + ": line-carry stencil pass"),
    ("--pmat", "auto", TRI + ": materialized-p split pass (irregular sparsity)"),
    ("--fused-reduce", "auto", TRI + ": in-kernel reduction (one kernel per iteration)"),
    ("--halo-mode", "auto", "auto | window | allgather"),
    ("--no-overlap", None, "halo on the compute stream (no interior / boundary split)"),
    ("--no-graph", None, "eager iterations (no hipGraph)"),
    ("--force-comm", None, "RCCL collectives also with one rank"),
    ("--comm", "single", "single (default): one communicator, one stream order | dual: reduce + halo communicators (halo on a side stream)"),
    ("--blocks-per-cu", "0", "SpMV grid, blocks per CU (0 = auto)"),
    ("--reserve-cus", "0", "CUs withheld from the compute stream (32 = one per shader engine) so collectives start beside the pass"),
    ("--spmv-variant", "-1", "CSR engine: 0 LDS tiles, 1 direct, 2 CSR-vector, 3 direct nt, 4 row-length adaptive; -1 auto"),
    # P > 1 transports (the solver's transport probe picks at the first reset)
    ("--halo-transport", "auto", "auto: the neighbours' halo buffers mapped (the lean carries read their ghost lines "
                                 "in-kernel) | rccl: RCCL's send/recv only"),
    ("--allreduce", "auto", "auto: IPC mailboxes mapped next to RCCL, the probe keeps the faster correct one | rccl | ipc"),
    ("--transport-probe", "auto", "auto | off: time the pulled vs exchanged halo and the two all-reduces at setup"),
    ("--rehearse-ranks", None, "--gpus P ranks all on GPU 0, the real P-rank recurrence (native: threads over an "
                               "in-process communicator; python: processes over IPC mailboxes and copy engines)"),
    # aux subsystems
    ("--checkpoint", None, "PREFIX of per-rank checkpoint files"),
    ("--checkpoint-every", "0", "write a checkpoint every ~K iterations"),
    ("--resume", None, "PREFIX: continue from a checkpoint"),
    ("--inject-nan-at", "-1", "fault injection: NaN into r at iteration K"),
    # output
    ("--print-x", "auto", "auto | yes | no (auto: n <= 1000)"),
    ("--report", "text", "text | json"),
    ("--verify", None, "also compute the true residual ||b - A x||"),
]


def tri(v: str) -> int:
    """auto|on|off (or -1|1|0) -> -1|1|0, the native parser's mapping."""
    v = str(v).lower()
    if v in ("auto", "-1"):
        return -1
    if v in ("on", "1", "yes"):
        return 1
    if v in ("off", "0", "no"):
        return 0
    raise ValueError(f"expected auto|on|off, got {v!r}")


def recurrence(v: str) -> int:
    v = str(v).lower()
    if v in ("auto", "-1"):
        return -1
    if v in ("single", "fused1", "1"):
        return 1
    if v in ("two", "0"):
        return 0
    if v in ("pipelined", "2"):
        return 2
    raise ValueError(f"expected auto|two|single|pipelined, got {v!r}")
