"""The variable-coefficient Poisson family (``coef=1``, problem.hpp): a seeded random conductivity
field, harmonic-mean face coefficients.  CPU checks of the generator (the reference takes arbitrary
stencil values, CUDACG.cu:93-117): symmetric bit for bit, SPD, the 5-/7-pt pattern and nnz of the
constant family, every value a pure function of the global row, the CPU oracle converging on it."""
import numpy as np
import pytest
import scipy.sparse as sp


@pytest.mark.parametrize("problem,n", [("poisson2d", 12), ("poisson3d", 6)])
def test_varcoef_symmetric_spd_same_pattern(mcg, problem, n):
    v = mcg.make_problem(problem, n=n, coef=1)
    c = mcg.make_problem(problem, n=n)
    A, B = mcg.models.to_scipy(v), mcg.models.to_scipy(c)
    assert A.nnz == B.nnz == c.nnz
    assert (A != A.T).nnz == 0  # exactly symmetric (face values from the ordered pair)
    np.testing.assert_array_equal(A.indices, B.indices)
    np.testing.assert_array_equal(A.indptr, B.indptr)
    assert np.linalg.eigvalsh(A.toarray()).min() > 0
    off = (A - sp.diags(A.diagonal())).tocsr()
    off.eliminate_zeros()
    assert (off.data < 0).all()
    # diagonally dominant: a_ii = sum of the face conductivities >= sum |a_ij| (boundary faces add)
    assert (A.diagonal() - np.abs(off).sum(axis=1).A1 >= -1e-12).all()
    assert len(np.unique(off.data)) > A.shape[0]  # far beyond the c8 / dia4 value tables


def test_varcoef_coefficient_range_and_seed(mcg):
    A = mcg.models.to_scipy(mcg.make_problem("poisson2d", n=64, coef=1, seed=7))
    A2 = mcg.models.to_scipy(mcg.make_problem("poisson2d", n=64, coef=1, seed=8))
    off = (A - sp.diags(A.diagonal())).tocsr()
    off.eliminate_zeros()
    k = -off.data
    assert k.min() >= 0.1 - 1e-12 and k.max() <= 10.0
    assert (A != A2).nnz > 0


def test_varcoef_partition_independent_host_rows(mcg):
    """A rank's host rows hold the global rows' values (every value a function of the global index)."""
    spec = mcg.make_problem("poisson2d", n=32, coef=1)
    A = mcg.models.to_scipy(spec).tocsr()
    rp, cols, vals = mcg.models.host_csr(spec, 4, 2)
    rows = len(rp) - 1
    assert rows == 32 * 32 // 4 and rp[-1] == len(vals)
    lo = 2 * rows
    for i in (0, 5, rows - 1):
        g = A.data[A.indptr[lo + i]:A.indptr[lo + i + 1]]
        np.testing.assert_array_equal(np.asarray(vals[rp[i]:rp[i + 1]]), g)


def test_varcoef_cpu_oracle_converges_and_names(mcg):
    spec = mcg.make_problem("poisson2d", n=48, coef=1, rhs="random")
    C = mcg.native()
    out = C.cpu_cg(spec.native(), C.CgOptions(maxit=4000, tol=1e-9))
    assert out["converged"]
    import scipy.sparse.linalg as sla
    A = mcg.models.to_scipy(spec)
    b = np.asarray(out["b"]) if "b" in out else None
    if b is not None:
        assert np.linalg.norm(b - A @ np.asarray(out["x"])) < 1e-8
    assert spec.native().name == "poisson2d-varcoef"
    assert mcg.make_problem("poisson3d", n=4, coef=1).native().name == "poisson3d-varcoef"
    with pytest.raises(Exception):
        mcg.make_problem("randspd", rows=100, band=4, coef=1).native()


def test_plane_carry_run_count_fills_rounds(mcg):
    """kern::carry3_runs (the 3-D plane carry's runs per job column, setup's choice): 512^3 with all
    256 CUs keeps one run (one job per block); 224 CUs (reserve_cus = 32) take 7 runs, whose 1792
    jobs fill 8 rounds exactly instead of 256 jobs running a second round for 32 blocks; a grid
    with fewer jobs than blocks splits its planes (384^3: 144 jobs per run)."""
    k = mcg.native().kernels
    assert k.carry3_runs(256, 256, 512) == 1
    assert k.carry3_runs(224, 256, 512) == 7
    assert k.carry3_runs(256, 64, 256) == 4  # the old rule (blocks / jobs) where it already fit
    r = k.carry3_runs(256, 144, 384)
    rounds = -(-144 * r // 256)
    assert r > 1 and rounds * (-(-384 // r) + 3) < 384 + 3
    assert k.carry3_runs(256, 8, 64) <= 16  # runs keep >= 4 planes


def test_plane_carry_runs_past_2_29_rows_stay_within_4_gib(mcg):
    """Past 2^29 rows a lean plane-carry run keeps its planes -3 .. end + 4 within 4 GiB of one 64-bit
    base (per-run bases; bases moved along the run spilled 60 VGPRs and ran at half rate): carry3_runs'
    max_chunk caps the planes per run -- 1024^3 (8 MiB planes) at most 504, 832^3 at most 767."""
    k = mcg.native().kernels
    for n, cap in ((1024, (1 << 32) // (1024 * 1024 * 8) - 8), (832, (1 << 32) // (832 * 832 * 8) - 8)):
        jpr = (n // 16) * (n // 64)  # jobs per run of the kw = 16 plane carry
        r = k.carry3_runs(256, jpr, n, cap)
        assert -(-n // r) <= cap, (n, r, cap)
        assert k.carry3_runs(256, jpr, n) <= r  # the cap only ever adds runs
    assert k.carry3_runs(256, 256, 512, 0) == k.carry3_runs(256, 256, 512)
