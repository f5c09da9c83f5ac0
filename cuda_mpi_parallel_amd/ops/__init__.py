"""Torch-tensor front end of the hand-written gfx950 kernels.

Every op runs the native HIP kernel from ``csrc/gpu/*.hip`` on the current torch
HIP stream; there is no PyTorch fallback — an op fails loudly if its input is not
a device tensor or if the native extension is missing.  These are the unfused
building blocks of the reference's per-iteration sequence (cuSPARSE SpMV,
cuBLAS dot/axpy/scal, CUDACG.cu:288-347); the solver itself uses the fused
kernels (see ``csrc/gpu/cg_kernels.hip``).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import native

_K = None


def _k():
    global _K
    if _K is None:
        _K = native().kernels
    return _K


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _req(t: torch.Tensor, dtype: torch.dtype, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise RuntimeError(f"{name}: expected a HIP device tensor (these ops have no CPU path)")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected dtype {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    return t


def spmv_csr(rowptr: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, x: torch.Tensor,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = A x for a CSR matrix (int32 or int64 row pointers, int32 columns, fp64 values),
    LDS-staged 256-row tiles."""
    if rowptr.dtype not in (torch.int32, torch.int64):
        raise TypeError("rowptr must be int32 or int64")
    _req(rowptr, rowptr.dtype, "rowptr")
    _req(cols, torch.int32, "cols")
    _req(vals, torch.float64, "vals")
    _req(x, torch.float64, "x")
    n = rowptr.numel() - 1
    if cols.numel() != vals.numel():
        raise ValueError("cols/vals length mismatch")
    # the LDS stager reads 16-B chunks that can straddle the last entry: pad to a multiple of 4
    if cols.numel() % 4:
        pad = 4 - cols.numel() % 4
        cols = torch.cat([cols, cols.new_zeros(pad)])
        vals = torch.cat([vals, vals.new_zeros(pad)])
    y = out if out is not None else torch.empty(n, dtype=torch.float64, device=x.device)
    _req(y, torch.float64, "out")
    _k().spmv_csr(rowptr.data_ptr(), rowptr.dtype == torch.int64, cols.data_ptr(), vals.data_ptr(), n,
                  x.data_ptr(), y.data_ptr(), _stream())
    return y


def csr_to_sell(rowptr: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor
                ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """CSR -> SELL-64 (slice_ptr int64, cols int32, vals fp64); padding = (own row, 0.0)."""
    rp64 = _req(rowptr.to(torch.int64), torch.int64, "rowptr")
    _req(cols, torch.int32, "cols")
    _req(vals, torch.float64, "vals")
    n = rp64.numel() - 1
    ns = (n + 63) // 64
    sp = torch.zeros(ns + 1, dtype=torch.int64, device=rp64.device)
    _k().sell_slice_widths(rp64.data_ptr(), n, sp.data_ptr(), _stream())
    sp[1:] = torch.cumsum(sp[1:], 0)
    total = int(sp[-1].item())
    scols = torch.empty(total, dtype=torch.int32, device=rp64.device)
    svals = torch.empty(total, dtype=torch.float64, device=rp64.device)
    _k().csr_to_sell(rp64.data_ptr(), cols.data_ptr(), vals.data_ptr(), n, sp.data_ptr(), scols.data_ptr(),
                     svals.data_ptr(), _stream())
    return sp, scols, svals


def spmv_sell(slice_ptr: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n_rows: int, x: torch.Tensor,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = A x for SELL-64 storage (one wave per 64-row slice, column-major entries)."""
    _req(slice_ptr, torch.int64, "slice_ptr")
    _req(cols, torch.int32, "cols")
    _req(vals, torch.float64, "vals")
    _req(x, torch.float64, "x")
    y = out if out is not None else torch.empty(n_rows, dtype=torch.float64, device=x.device)
    _k().spmv_sell(slice_ptr.data_ptr(), cols.data_ptr(), vals.data_ptr(), n_rows, x.data_ptr(), y.data_ptr(),
                   _stream())
    return y


def sell_compress_c8(slice_ptr: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n_rows: int
                     ) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """SELL-64 -> SELL-64/c8: one byte per stored entry indexing a table of distinct
    (value, column offset) pairs (csrc/gpu/dict.hip).  Returns (codes uint8, dict float64 [k, 2])
    or None when the matrix has more than 256 distinct pairs."""
    _req(slice_ptr, torch.int64, "slice_ptr")
    _req(cols, torch.int32, "cols")
    _req(vals, torch.float64, "vals")
    r = _k().sell_dict_build(slice_ptr.data_ptr(), cols.data_ptr(), vals.data_ptr(), n_rows, _stream())
    if r is None:
        return None
    d, nv, nd = r
    dict_t = torch.from_numpy(d).to(vals.device)
    codes = torch.empty(vals.numel(), dtype=torch.uint8, device=vals.device)
    _k().sell_to_c8(slice_ptr.data_ptr(), cols.data_ptr(), vals.data_ptr(), n_rows, dict_t.data_ptr(), nv, nd,
                    codes.data_ptr(), _stream())
    return codes, dict_t


def spmv_sell_c8(slice_ptr: torch.Tensor, codes: torch.Tensor, dict_t: torch.Tensor, n_rows: int, x: torch.Tensor,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = A x for SELL-64/c8 storage (codes from :func:`sell_compress_c8`)."""
    _req(slice_ptr, torch.int64, "slice_ptr")
    _req(codes, torch.uint8, "codes")
    _req(dict_t, torch.float64, "dict")
    _req(x, torch.float64, "x")
    if dict_t.dim() != 2 or dict_t.shape[1] != 2 or dict_t.shape[0] > 256:
        raise ValueError("dict must be [k <= 256, 2]")
    y = out if out is not None else torch.empty(n_rows, dtype=torch.float64, device=x.device)
    _k().spmv_sell_c8(slice_ptr.data_ptr(), codes.data_ptr(), dict_t.data_ptr(), dict_t.shape[0], n_rows,
                      x.data_ptr(), y.data_ptr(), _stream())
    return y


def dot(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Fixed-order two-stage dot product (block partials -> one block); returns a 1-element tensor."""
    _req(a, torch.float64, "a")
    _req(b, torch.float64, "b")
    if a.numel() != b.numel():
        raise ValueError("length mismatch")
    n = a.numel()
    grid = _k().grid_for((n + 1) // 2, 256, 8)
    partials = torch.empty(grid, dtype=torch.float64, device=a.device)
    out = torch.empty(1, dtype=torch.float64, device=a.device)
    _k().dot_partials(a.data_ptr(), b.data_ptr(), n, partials.data_ptr(), grid, _stream())
    _k().sum_partials(partials.data_ptr(), grid, out.data_ptr(), _stream())
    return out


def axpy(alpha: float, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """y += alpha * x (in place)."""
    _req(x, torch.float64, "x")
    _req(y, torch.float64, "y")
    _k().axpy(float(alpha), x.data_ptr(), y.data_ptr(), y.numel(), _stream())
    return y


def xpby(x: torch.Tensor, beta: float, y: torch.Tensor) -> torch.Tensor:
    """y = x + beta * y (in place) — the reference's SCAL+AXPY pair (CUDACG.cu:342-347) in one pass."""
    _req(x, torch.float64, "x")
    _req(y, torch.float64, "y")
    _k().xpby(x.data_ptr(), float(beta), y.data_ptr(), y.numel(), _stream())
    return y


def generate_csr(spec, row_begin: int = 0, n: Optional[int] = None, device: str = "cuda"
                 ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """On-device generation of rows [row_begin, row_begin+n) with GLOBAL column indices."""
    ns = spec.native() if hasattr(spec, "native") else spec
    n = int(ns.n_rows) - row_begin if n is None else n
    rp = torch.empty(n + 1, dtype=torch.int64, device=device)
    s = _stream()
    _k().gen_rowlen(ns, row_begin, n, rp.data_ptr(), s)
    tmp = torch.empty(_k().scan_tmp_elems(n), dtype=torch.int64, device=device)
    _k().scan_inclusive_i64(rp.data_ptr() + 8, n, tmp.data_ptr(), s)
    nnz = int(rp[-1].item())
    cols = torch.empty(nnz + 8, dtype=torch.int32, device=device)
    vals = torch.empty(nnz + 8, dtype=torch.float64, device=device)
    _k().gen_fill(ns, row_begin, n, 0, 0, rp.data_ptr(), cols.data_ptr(), vals.data_ptr(), s)
    return rp, cols[:nnz], vals[:nnz]


def generate_rhs(spec, row_begin: int = 0, n: Optional[int] = None, device: str = "cuda") -> torch.Tensor:
    ns = spec.native() if hasattr(spec, "native") else spec
    n = int(ns.n_rows) - row_begin if n is None else n
    b = torch.empty(n, dtype=torch.float64, device=device)
    _k().gen_rhs(ns, row_begin, n, b.data_ptr(), _stream())
    return b


__all__ = ["spmv_csr", "spmv_sell", "csr_to_sell", "sell_compress_c8", "spmv_sell_c8", "dot", "axpy", "xpby", "generate_csr", "generate_rhs"]
