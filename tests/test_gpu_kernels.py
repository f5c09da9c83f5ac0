"""GPU numerics of the hand-written kernels vs plain PyTorch / NumPy fp64 references."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rand_csr(n, max_len, seed, long_rows=False):
    g = np.random.default_rng(seed)
    lens = g.integers(0, max_len + 1, size=n)
    if long_rows:
        lens[:: max(1, n // 7)] = 3000  # rows spanning several 2048-nnz LDS chunks
    rowptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    nnz = int(rowptr[-1])
    cols = g.integers(0, n, size=nnz).astype(np.int32)
    vals = g.standard_normal(nnz)
    return rowptr, cols, vals


def _ref_spmv(rowptr, cols, vals, x):
    n = len(rowptr) - 1
    rows = np.repeat(np.arange(n), np.diff(rowptr))
    return np.bincount(rows, weights=vals * x[cols], minlength=n)


@pytest.mark.parametrize("n,max_len,long_rows,idx64", [
    (1, 3, False, False), (63, 5, False, False), (1000, 7, False, True), (5000, 12, True, False),
    (70000, 5, False, False)])
def test_spmv_csr_matches_reference(mcg, n, max_len, long_rows, idx64):
    rowptr, cols, vals = _rand_csr(n, max_len, seed=n, long_rows=long_rows)
    x = np.random.default_rng(1).standard_normal(n)
    d = "cuda"
    rp = torch.tensor(rowptr, device=d, dtype=torch.int64 if idx64 else torch.int32)
    y = mcg.ops.spmv_csr(rp, torch.tensor(cols, device=d), torch.tensor(vals, device=d), torch.tensor(x, device=d))
    torch.cuda.synchronize()
    ref = _ref_spmv(rowptr, cols, vals, x)
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=1e-12, atol=1e-12)


def test_spmv_sell_matches_csr(mcg):
    rowptr, cols, vals = _rand_csr(3001, 9, seed=7)
    x = np.random.default_rng(2).standard_normal(3001)
    d = "cuda"
    rp, c, v = (torch.tensor(rowptr, device=d), torch.tensor(cols, device=d), torch.tensor(vals, device=d))
    sp, sc, sv = mcg.ops.csr_to_sell(rp, c, v)
    y = mcg.ops.spmv_sell(sp, sc, sv, 3001, torch.tensor(x, device=d))
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.cpu().numpy(), _ref_spmv(rowptr, cols, vals, x), rtol=1e-12, atol=1e-12)


def test_spmv_sell_c8_matches_fp64_reference(mcg):
    """Dictionary-coded SELL (1 byte per entry) on a 5-pt stencil with a ragged tail slice
    vs a plain fp64 PyTorch SpMV; a random matrix (too many distinct values) is refused."""
    spec = mcg.make_problem("poisson2d", n=45)  # 2025 rows: last slice has 41 live rows
    rowptr, cols, vals = mcg.native().host_csr(spec.native(), 1, 0)
    n = len(rowptr) - 1
    d = "cuda"
    rp, c, v = (torch.tensor(rowptr, device=d), torch.tensor(cols, device=d), torch.tensor(vals, device=d))
    sp, sc, sv = mcg.ops.csr_to_sell(rp, c, v)
    codes, dict_t = mcg.ops.sell_compress_c8(sp, sc, sv, n)
    assert codes.dtype == torch.uint8 and dict_t.shape[0] <= 256
    x = torch.tensor(np.random.default_rng(3).standard_normal(n), device=d)
    y = mcg.ops.spmv_sell_c8(sp, codes, dict_t, n, x)
    ref = torch.sparse_csr_tensor(torch.tensor(rowptr), torch.tensor(cols), torch.tensor(vals), (n, n)) @ x.cpu()
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.cpu().numpy(), ref.numpy(), rtol=1e-13, atol=1e-13)
    # bit-identical to the uncompressed SELL kernel (same entries, same order)
    assert torch.equal(y, mcg.ops.spmv_sell(sp, sc, sv, n, x))
    rowptr, cols, vals = _rand_csr(3001, 9, seed=7)
    rp, c, v = (torch.tensor(rowptr, device=d), torch.tensor(cols, device=d), torch.tensor(vals, device=d))
    sp, sc, sv = mcg.ops.csr_to_sell(rp, c, v)
    assert mcg.ops.sell_compress_c8(sp, sc, sv, 3001) is None


@pytest.mark.parametrize("n", [1, 2, 3, 1001, 1 << 20])
def test_dot_axpy_xpby(mcg, n):
    g = torch.Generator().manual_seed(n)
    a = torch.randn(n, dtype=torch.float64, generator=g)
    b = torch.randn(n, dtype=torch.float64, generator=g)
    ad, bd = a.cuda(), b.cuda()
    got = mcg.ops.dot(ad, bd).item()
    assert abs(got - float(a @ b)) <= 1e-10 * (1 + float(a.abs() @ b.abs()))
    y = bd.clone()
    mcg.ops.axpy(-0.37, ad, y)
    torch.testing.assert_close(y.cpu(), b - 0.37 * a, rtol=1e-14, atol=1e-14)
    y = bd.clone()
    mcg.ops.xpby(ad, 1.7, y)
    torch.testing.assert_close(y.cpu(), a + 1.7 * b, rtol=1e-14, atol=1e-14)


@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=37)), ("poisson3d", dict(n=11)),
                                         ("randspd", dict(rows=5000, band=50, density=0.3)), ("demo", {})])
def test_device_generator_matches_host(mcg, problem, kw):
    spec = mcg.make_problem(problem, **kw)
    rp, c, v = mcg.ops.generate_csr(spec)
    hrp, hc, hv = mcg.models.host_csr(spec)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(rp.cpu().numpy(), hrp)
    np.testing.assert_array_equal(c.cpu().numpy(), hc)
    np.testing.assert_array_equal(v.cpu().numpy(), hv)
    b = mcg.ops.generate_rhs(spec)
    np.testing.assert_array_equal(b.cpu().numpy(), mcg.models.rhs(spec))
