"""User matrices (problem kind ``csr``): the reference's own input form, a CSR triple
(CUDACG.cu:93-117) handed to the generic SpMV (CUDACG.cu:213-216).  CPU paths: host CSR,
Matrix Market reader, partition / ghost plan from the actual columns, CPU reference solve,
virtual ranks, gloo processes, both CLIs."""
import os
import subprocess
import sys

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp
import torch.multiprocessing as mp

from test_dist_gloo import _free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO_MTX = """%%MatrixMarket matrix coordinate real symmetric
% the reference's 3x3 system (CUDACG.cu:74-117), lower triangle
3 3 4
1 1 3
2 2 2
3 1 2
3 3 1
"""


def _spd(n=400, density=0.01, seed=3, shift=None):
    A = sp.random(n, n, density=density, random_state=seed, format="csr")
    A = A + A.T
    d = np.asarray(abs(A).sum(axis=1)).ravel() + 1.0
    return (A + sp.diags(d if shift is None else shift)).tocsr()


def _opts(C, **kw):
    o = C.CgOptions(maxit=kw.pop("maxit", 2000), tol=kw.pop("tol", 1e-10))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def test_reference_demo_through_csr_path(mcg, C, tmp_path):
    f = tmp_path / "demo.mtx"
    f.write_text(DEMO_MTX)
    p = mcg.csr_problem(str(f), b=np.array([3.5, 1.5, 2.0]))
    r = C.cpu_cg(p.native(), C.CgOptions())
    assert "".join("%f\n" % v for v in r["x"]) == "0.500000\n0.750000\n1.000000\n"
    assert r["iterations"] == 3


def test_matrix_market_reader_matches_scipy(mcg, tmp_path):
    A = _spd(60, 0.05)
    f = tmp_path / "a.mtx"
    scipy.io.mmwrite(str(f), A, symmetry="symmetric")
    H = mcg.native().HostMatrix.read_mtx(str(f))
    assert H.n == 60 and H.nnz == A.nnz and H.symmetric()
    p = mcg.models.CsrProblem(H)
    B = mcg.models.to_scipy(p)
    assert abs(B - A).max() < 1e-12
    # general storage with a duplicate entry (summed), pattern field, errors
    g = tmp_path / "g.mtx"
    g.write_text("%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1.5\n1 1 0.5\n2 2 4\n")
    H = mcg.native().HostMatrix.read_mtx(str(g))
    assert H.nnz == 2
    assert np.allclose(mcg.models.to_scipy(mcg.models.CsrProblem(H)).toarray(), [[2, 0], [0, 4]])
    bad = tmp_path / "bad.mtx"
    bad.write_text("%%MatrixMarket matrix coordinate real general\n2 3 1\n1 1 1\n")
    with pytest.raises(Exception, match="matrix read failed"):
        mcg.native().HostMatrix.read_mtx(str(bad))


def test_host_matrix_validates_and_sorts(mcg):
    H = mcg.native().HostMatrix(np.array([0, 2, 3]), np.array([1, 0, 1]), np.array([2.0, 1.0, 3.0]))
    assert H.bandwidth == 1
    A = mcg.models.to_scipy(mcg.models.CsrProblem(H)).toarray()
    assert np.array_equal(A, [[1.0, 2.0], [0.0, 3.0]])
    with pytest.raises(Exception):
        mcg.native().HostMatrix(np.array([0, 1]), np.array([5]), np.array([1.0]))


def test_cpu_solve_matches_scipy(mcg, C):
    A = _spd()
    b = np.random.default_rng(0).standard_normal(A.shape[0])
    p = mcg.csr_problem(A, b=b)
    r = C.cpu_cg(p.native(), _opts(C))
    assert r["converged"]
    np.testing.assert_allclose(r["x"], sp.linalg.spsolve(A.tocsc(), b), rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("kind", ["unstructured", "banded"])
def test_virtual_ranks_match(mcg, C, world, kind):
    A = _spd() if kind == "unstructured" else sp.diags([-1, -1, 4, -1, -1], [-7, -1, 0, 1, 7], shape=(500, 500)).tocsr()
    p = mcg.csr_problem(A)
    L = mcg.parallel.layout(p, world, 0)
    assert L.allgather == (kind == "unstructured")
    if kind == "banded":  # ghost ranges from the actual columns: +-7 rows per side
        assert all(c <= 7 for _, _, c in L.recvs)
    a = C.cpu_cg(p.native(), _opts(C, maxit=500))
    b = C.cpu_cg_partitioned(p.native(), world, _opts(C, maxit=500))
    assert abs(a["iterations"] - b["iterations"]) <= 1
    np.testing.assert_allclose(b["x"], a["x"], rtol=1e-9, atol=1e-12)


def test_rcm_reorder_gives_window_layout_and_same_solution(mcg, C):
    n = 30
    A = sp.diags([-1, -1, 4, -1, -1], [-n, -1, 0, 1, n], shape=(n * n, n * n)).tocsr()
    perm = np.random.default_rng(1).permutation(n * n)
    Ap = A[perm][:, perm].tocsr()  # a scrambled 2-D Laplacian: unstructured as stored
    b = np.ones(n * n)
    plain = mcg.csr_problem(Ap, b=b)
    rcm = mcg.csr_problem(Ap, b=b, reorder="rcm")
    assert mcg.parallel.layout(plain, 4, 1).allgather
    assert not mcg.parallel.layout(rcm, 4, 1).allgather
    x1 = C.cpu_cg(plain.native(), _opts(C))["x"]
    x2 = rcm.unpermute(C.cpu_cg(rcm.native(), _opts(C))["x"])
    np.testing.assert_allclose(x2, x1, rtol=1e-8, atol=1e-10)


def _worker(rank, world, port, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import cuda_mpi_parallel_amd as mcg
    from cuda_mpi_parallel_amd.parallel.cpu_ref import cpu_cg_distributed, gather_x

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = cpu_cg_distributed(mcg.csr_problem(path), maxit=2000, tol=1e-10)
        x = gather_x(out)
        if rank == 0:
            q.put((out["iterations"], x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_processes_each_read_the_file(mcg, C, world, tmp_path):
    f = tmp_path / "a.mtx"
    scipy.io.mmwrite(str(f), _spd(300, 0.02))
    ref = C.cpu_cg(mcg.csr_problem(str(f)).native(), _opts(C))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(f), q)) for r in range(world)]
    for p in procs:
        p.start()
    its, x = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert abs(its - ref["iterations"]) <= 1
    np.testing.assert_allclose(x, ref["x"], rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("cli", ["native", "python"])
def test_cli_matrix_flag_golden(mcg, tmp_path, cli):
    f = tmp_path / "demo.mtx"
    f.write_text(DEMO_MTX)
    b = tmp_path / "b.txt"
    b.write_text("3.5\n1.5\n2.0\n")
    head = [mcg.cli_path()] if cli == "native" else [sys.executable, "-m", "cuda_mpi_parallel_amd"]
    p = subprocess.run(head + ["--device", "cpu", "--matrix", str(f), "--rhs-file", str(b)], capture_output=True,
                       text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout == "0.500000\n0.750000\n1.000000\nSuccess\n"


def test_solve_helper_takes_a_matrix(mcg):
    A = _spd(300, 0.02)
    b = np.arange(300, dtype=float) / 300.0
    for reorder in (None, "rcm"):
        r = mcg.solve(matrix=A, b=b, device="cpu", tol=1e-10, reorder=reorder)
        np.testing.assert_allclose(r["x"], sp.linalg.spsolve(A.tocsc(), b), rtol=1e-8, atol=1e-10)


@pytest.mark.parametrize("dim", [2, 3])
def test_stencil_detection_and_line_partition(mcg, C, dim):
    """A user matrix whose column offsets are {0, +-1, +-n} (2-D) or also +-n^2 (3-D) is recognised
    as a grid stencil; a P-rank partition then cuts at whole lines / planes.  Other matrices keep
    line = 0 and the nnz-balanced partition."""
    n = 16
    T = sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(n, n))
    I = sp.identity(n)
    A = (sp.kron(I, T) + sp.kron(T, I)) if dim == 2 else (
        sp.kron(sp.kron(I, I), T) + sp.kron(sp.kron(I, T), I) + sp.kron(sp.kron(T, I), I))
    p = mcg.csr_problem(A.tocsr())
    g = n if dim == 2 else n * n
    assert p.matrix.stencil_line == n and p.matrix.stencil_plane == (0 if dim == 2 else g)
    for world in (2, 3, 5):
        offs = C.partition_rows(p.native(), world, 0)
        assert all(o % g == 0 for o in offs), offs
    q = mcg.csr_problem(_spd())
    assert q.matrix.stencil_line == 0 and q.matrix.stencil_plane == 0
    # a matrix with the offsets but rows that are not whole lines: no stencil
    B = sp.diags([-1.0, -1.0, 4.0, -1.0, -1.0], [-n, -1, 0, 1, n], shape=(n * n - 3, n * n - 3)).tocsr()
    assert mcg.csr_problem(B).matrix.stencil_line == 0


def test_read_vector_formats(C, tmp_path):
    """--rhs-file: a Matrix Market `array` vector (size line checked), plain one-value-per-line text,
    and a clear refusal of a `coordinate` file (whose "i j v" lines would otherwise be read as b)."""
    a = tmp_path / "a.mtx"
    a.write_text("%%MatrixMarket matrix array real general\n% comment\n3 1\n3.5\n1.5\n2.0\n")
    assert list(C.read_vector(str(a))) == [3.5, 1.5, 2.0]
    t = tmp_path / "b.txt"
    t.write_text("1\n2\n")
    assert list(C.read_vector(str(t))) == [1.0, 2.0]
    c = tmp_path / "c.mtx"
    c.write_text("%%MatrixMarket matrix coordinate real general\n3 1 2\n1 1 3.5\n3 1 2.0\n")
    with pytest.raises(Exception, match="array"):
        C.read_vector(str(c))
    s = tmp_path / "s.mtx"
    s.write_text("%%MatrixMarket matrix array real general\n4 1\n1\n2\n3\n")
    with pytest.raises(Exception, match="size line"):
        C.read_vector(str(s))
