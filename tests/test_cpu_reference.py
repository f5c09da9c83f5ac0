"""CPU reference path (BASELINE.json config 1) and problem-family numerics; no GPU."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla


def test_demo_recurrence_matches_reference_replay(C):
    """The reference recurrence on the 3x3 system: 3 steps, ||r|| = 0.807, 0.167, ~8e-15."""
    out = C.cpu_cg(C.ProblemSpec("demo"), C.CgOptions())
    assert out["iterations"] == 3 and out["converged"]
    h = out["rnorm_history"]
    np.testing.assert_allclose(h[:2], [0.807385477, 0.167342799], rtol=1e-8)
    assert h[2] < 1e-13
    assert "".join("%f\n" % v for v in out["x"]) == "0.500000\n0.750000\n1.000000\n"


@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=48)), ("poisson3d", dict(n=12)),
                                         ("randspd", dict(rows=3000, band=25, density=0.4))])
def test_cpu_cg_matches_scipy(mcg, C, problem, kw):
    spec = mcg.make_problem(problem, **kw)
    A = mcg.models.to_scipy(spec)
    b = mcg.models.rhs(spec)
    out = C.cpu_cg(spec.native(), C.CgOptions(maxit=5000, tol=1e-9))
    x_ref, info = spla.cg(A, b, rtol=0.0, atol=1e-12, maxiter=5000)
    assert info == 0 and out["converged"]
    np.testing.assert_allclose(out["x"], x_ref, rtol=1e-6, atol=1e-8 * np.abs(x_ref).max())
    assert np.linalg.norm(b - A @ out["x"]) < 1e-8


def test_maxit_exhaustion_is_silent_success(C):
    """Reaching maxit still returns x (reference prints x and Success regardless, CUDACG.cu:269,365)."""
    spec = C.ProblemSpec("poisson2d", 64, rhs="random")
    out = C.cpu_cg(spec, C.CgOptions(maxit=5, tol=1e-7))
    assert out["iterations"] == 5 and not out["converged"] and len(out["x"]) == 64 * 64


def test_indefinite_demo_no_abort_on_negative_curvature(mcg):
    A = mcg.models.to_scipy(mcg.make_problem("demo")).toarray()
    assert np.linalg.eigvalsh(A).min() < 0  # p^T A p < 0 happens in step 3 and must not abort


@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=30)), ("poisson3d", dict(n=10)),
                                         ("randspd", dict(rows=2000, band=20, density=0.3)), ("demo", {})])
def test_virtual_ranks_match_single_process(mcg, C, world, problem, kw):
    """P virtual ranks with the GPU solver's partition + halo plan == one process (to rounding)."""
    spec = mcg.make_problem(problem, **kw)
    o = C.CgOptions(maxit=500, tol=1e-9)
    a = C.cpu_cg(spec.native(), o)
    b = C.cpu_cg_partitioned(spec.native(), world, o)
    assert abs(a["iterations"] - b["iterations"]) <= 1
    np.testing.assert_allclose(b["x"], a["x"], rtol=1e-7, atol=1e-9 * (1 + np.abs(a["x"]).max()))


def test_problem_matrices_symmetric_and_spd(mcg):
    for spec in [mcg.make_problem("poisson2d", n=9), mcg.make_problem("poisson3d", n=5),
                 mcg.make_problem("randspd", rows=400, band=15, density=0.5)]:
        A = mcg.models.to_scipy(spec)
        assert abs(A - A.T).max() == 0
        assert np.linalg.eigvalsh(A.toarray()).min() > 0


def test_closed_form_nnz(mcg):
    for name, n in [("poisson2d", 16384), ("poisson3d", 512)]:
        spec = mcg.make_problem(name, n=n)
        assert spec.nnz == (5 * n * n - 4 * n if name == "poisson2d" else 7 * n ** 3 - 6 * n * n)
    assert mcg.make_problem("poisson2d", n=16384).nnz == 1_342_111_744
    assert mcg.make_problem("poisson3d", n=512).nnz == 937_951_232


def test_rhs_independent_of_partition(mcg):
    spec = mcg.make_problem("poisson2d", n=40)
    full = mcg.models.rhs(spec)
    parts = [mcg.models.rhs(spec, a, b) for a, b in [(0, 500), (500, 1111), (1111, 1600)]]
    np.testing.assert_array_equal(np.concatenate(parts), full)
    assert 0.0 <= full.min() and full.max() < 1.0 and full.std() > 0.2


def test_relative_tolerance_option(mcg):
    """--rtol R stops on ||r|| < R ||b|| (the reference's comment says "relative", its code is absolute)."""
    C = mcg.native()
    spec = mcg.make_problem("poisson2d", n=64)
    bn = float(np.linalg.norm(mcg.models.rhs(spec)))
    o = C.CgOptions(maxit=2000, tol=1e-30)
    o.rtol = 1e-6
    r = C.cpu_cg(spec.native(), o)
    assert r["converged"] and r["rnorm"] < 1e-6 * bn
    o2 = C.CgOptions(maxit=2000, tol=1e-6 * bn)
    assert C.cpu_cg(spec.native(), o2)["iterations"] == r["iterations"]
    v = C.cpu_cg_partitioned(spec.native(), 3, o)
    assert abs(v["iterations"] - r["iterations"]) <= 1


def test_problem_aliases_and_nnz_per_row(mcg):
    s = mcg.make_problem("random-spd", rows=2000, band=40, nnz_per_row=17)
    assert s.problem == "randspd" and abs(s.density - 0.2) < 1e-12
