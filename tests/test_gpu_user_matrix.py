"""User CSR matrices on the GPU (problem kind ``csr``): the reference's input form
(CUDACG.cu:93-117) through every storage format and both recurrences, one GPU and P
in-process ranks (LocalComm) with window and all-gather ghost plans."""
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

DEMO = (np.array([0, 2, 3, 5]), np.array([0, 2, 1, 0, 2]), np.array([3.0, 2.0, 2.0, 2.0, 1.0]))


def _spd(n=3000, density=0.003, seed=5):
    A = sp.random(n, n, density=density, random_state=seed, format="csr")
    A = A + A.T
    return (A + sp.diags(np.asarray(abs(A).sum(axis=1)).ravel() + 1.0)).tocsr()


def _fd(n=40):  # a 2-D Laplacian given as a user matrix (dictionary codes apply)
    return sp.diags([-1, -1, 4, -1, -1], [-n, -1, 0, 1, n], shape=(n * n, n * n)).tocsr()


def test_reference_demo_csr_golden(mcg):
    p = mcg.csr_problem(DEMO, b=np.array([3.5, 1.5, 2.0]))
    out = mcg.CGSolver(p, format="csr").solve()
    assert mcg.utils.format_x(out["x_local"]) == "0.500000\n0.750000\n1.000000\n"
    assert out["iterations"] == 3 and out["converged"]


@pytest.mark.parametrize("fmt", ["csr", "sell", "sell16", "sellc8"])
@pytest.mark.parametrize("recurrence", [0, 1])
@pytest.mark.parametrize("which", ["unstructured", "laplacian"])
def test_user_matrix_matches_cpu(mcg, fmt, recurrence, which):
    A = _spd() if which == "unstructured" else _fd()
    b = np.random.default_rng(2).standard_normal(A.shape[0])
    p = mcg.csr_problem(A, b=b)
    C = mcg.native()
    cpu = C.cpu_cg(p.native(), C.CgOptions(maxit=2000, tol=1e-8))
    s = mcg.CGSolver(p, format=fmt, recurrence=recurrence, tol=1e-8, check_every=8)
    out = s.solve()
    assert out["converged"] and abs(out["iterations"] - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-6, atol=1e-7 * np.abs(cpu["x"]).max())
    np.testing.assert_allclose(A @ out["x_local"], b, atol=1e-6)
    if which == "laplacian" and fmt == "sellc8":
        assert s.info["format"] == "sell64-c8"  # 5 values x 5 offsets: one-byte codes


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("which", ["unstructured", "laplacian"])
@pytest.mark.parametrize("recurrence", [0, 1])
def test_user_matrix_local_ranks(mcg, world, which, recurrence):
    A = _spd() if which == "unstructured" else _fd()
    p = mcg.csr_problem(A)
    assert mcg.parallel.layout(p, world, 0).allgather == (which == "unstructured")
    C = mcg.native()
    cpu = C.cpu_cg(p.native(), C.CgOptions(maxit=2000, tol=1e-8))
    o = C.CgOptions(maxit=2000, tol=1e-8, format="sell", recurrence=recurrence, check_every=4)
    out = C.run_local_ranks(p.native(), o, world, 0, True)
    its = {r["iterations"] for r in out["ranks"]}
    assert len(its) == 1 and abs(its.pop() - cpu["iterations"]) <= 2
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-6, atol=1e-7 * np.abs(cpu["x"]).max())


def test_cli_matrix_on_gpu_golden(mcg, tmp_path):
    f = tmp_path / "demo.mtx"
    f.write_text("%%MatrixMarket matrix coordinate real symmetric\n3 3 4\n1 1 3\n2 2 2\n3 1 2\n3 3 1\n")
    b = tmp_path / "b.txt"
    b.write_text("3.5\n1.5\n2.0\n")
    p = subprocess.run([mcg.cli_path(), "--matrix", str(f), "--rhs-file", str(b)], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout == "0.500000\n0.750000\n1.000000\nSuccess\n"
