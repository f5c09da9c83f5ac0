"""Irregular-sparsity path on the CPU (BASELINE.json config 5): the wide random-SPD family
(candidate offsets spread over +-spread rows: multi-diagonal), the scrambled family P^T A P
(genuinely irregular), the all-gather ghost layout they select, and the CPU reference /
virtual-rank / gloo multi-process solves through that layout.

The reference solves one generic CSR matrix with cuSPARSE (CUDACG.cu:213-216, 288); any
sparsity must work, including columns spread over the whole matrix.
"""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_dist_gloo import _free_port

WIDE = dict(rows=3000, band=12, density=0.5, spread=3000)
SCRAMBLED = dict(rows=3000, band=12, density=0.5, scramble=1)


@pytest.mark.parametrize("n", [2, 3, 5, 64, 1000, 1023, 1024, 1025, 4097])
def test_scramble_permutation_is_a_bijection(mcg, n):
    """pi (Feistel + cycle walking) is a bijection of [0, n) and pi^-1 inverts it."""
    s = mcg.make_problem("randspd", rows=n, band=4, density=0.3, scramble=1).native()
    f = np.array([s.perm(i) for i in range(n)])
    g = np.array([s.perm(i, True) for i in range(n)])
    assert sorted(f.tolist()) == list(range(n))
    np.testing.assert_array_equal(g[f], np.arange(n))
    if n >= 1000:  # a random permutation: few fixed points, order destroyed
        assert (f == np.arange(n)).sum() < 10
        assert abs(np.corrcoef(f, np.arange(n))[0, 1]) < 0.1


def test_scrambled_is_permuted_base_and_irregular(mcg):
    """The scrambled matrix is exactly P^T A P of the base family: symmetric, strictly diagonally
    dominant, and unlike the multi-diagonal families no two rows share a column-offset set."""
    base = mcg.make_problem("randspd", rows=3000, band=12, density=0.5)
    spec = mcg.make_problem("randspd", **SCRAMBLED)
    A, B = mcg.models.to_scipy(spec), mcg.models.to_scipy(base)
    pi = np.array([spec.native().perm(i) for i in range(3000)])
    assert abs(A - B[pi][:, pi]).max() == 0 and A.nnz == B.nnz
    assert abs(A - A.T).max() == 0
    d = A.diagonal()
    assert (d > np.asarray(abs(A).sum(axis=1)).ravel() - d).all()
    A = A.tocsr()
    offsets = {tuple(sorted(A.indices[A.indptr[i]:A.indptr[i + 1]] - i)) for i in range(3000)}
    assert len(offsets) == 3000  # every row its own offset set (the wide family shares 2W offsets)
    W = mcg.models.to_scipy(mcg.make_problem("randspd", **WIDE)).tocsr()
    wide_offsets = set()
    for i in range(3000):
        wide_offsets.update((W.indices[W.indptr[i]:W.indptr[i + 1]] - i).tolist())
    assert len(wide_offsets) <= 2 * WIDE["band"] + 1
    lens = np.diff(A.indptr)
    assert lens.min() < lens.max()
    assert spec.native().bandwidth == 2999 and spec.native().name == "randspd-scrambled"


@pytest.mark.parametrize("world", [2, 3, 8])
def test_scrambled_virtual_ranks_match_single_process(mcg, C, world):
    """The scrambled family selects the all-gather layout; P virtual ranks reproduce P = 1."""
    spec = mcg.make_problem("randspd", **SCRAMBLED)
    assert all(mcg.parallel.layout(spec, world, r).allgather for r in range(world))
    o = C.CgOptions(maxit=500, tol=1e-9)
    a = C.cpu_cg(spec.native(), o)
    b = C.cpu_cg_partitioned(spec.native(), world, o)
    assert a["converged"] and abs(a["iterations"] - b["iterations"]) <= 1
    np.testing.assert_allclose(b["x"], a["x"], rtol=1e-9, atol=1e-12 * (1 + np.abs(a["x"]).max()))


def test_wide_randspd_is_symmetric_dominant_and_unstructured(mcg):
    spec = mcg.make_problem("randspd", **WIDE)
    A = mcg.models.to_scipy(spec).tocoo()
    assert abs(mcg.models.to_scipy(spec) - mcg.models.to_scipy(spec).T).max() == 0
    d = A.tocsr().diagonal()
    off = np.asarray(abs(A.tocsr()).sum(axis=1)).ravel() - d
    assert (d > off).all()  # strict diagonal dominance -> SPD
    span = np.abs(A.row - A.col)
    assert span.max() > WIDE["rows"] // 2  # columns reach across the matrix
    lens = np.diff(A.tocsr().indptr)
    assert lens.min() < lens.max()  # irregular row lengths
    assert spec.native().bandwidth == WIDE["spread"]


def test_wide_offsets_distinct_and_increasing(mcg):
    spec = mcg.make_problem("randspd", rows=100000, band=64, density=0.5, spread=90000)
    cols, _ = spec.native().row(50000)
    assert cols == sorted(set(cols))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_all_gather_layout_selected_and_consistent(mcg, world):
    spec = mcg.make_problem("randspd", **WIDE)
    Ls = [mcg.parallel.layout(spec, world, r) for r in range(world)]
    blk = Ls[0].block
    assert all(L.allgather for L in Ls) and blk % 64 == 0 and blk * world >= spec.n_rows
    for r, L in enumerate(Ls):
        assert L.own_off == r * blk and L.ext_len == world * blk and L.col_lo == 0
        assert L.interior_begin == L.interior_end  # no rows without remote columns
        assert sorted(p for p, _, _ in L.recvs) == [q for q in range(world) if q != r and Ls[q].n_local > 0]
    # a banded matrix keeps the column-window plan; the option forces either layout
    banded = mcg.make_problem("randspd", rows=3000, band=12, density=0.5)
    assert not mcg.parallel.layout(banded, world, 0).allgather
    assert mcg.parallel.layout(banded, world, 0, halo_mode=1).allgather
    assert not mcg.parallel.layout(spec, world, 0, halo_mode=0).allgather


@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("halo_mode", [-1, 0])
def test_virtual_ranks_wide_match_single_process(mcg, C, world, halo_mode):
    spec = mcg.make_problem("randspd", **WIDE)
    o = C.CgOptions(maxit=500, tol=1e-9)
    o.halo_mode = halo_mode
    a = C.cpu_cg(spec.native(), o)
    b = C.cpu_cg_partitioned(spec.native(), world, o)
    assert a["converged"] and abs(a["iterations"] - b["iterations"]) <= 1
    np.testing.assert_allclose(b["x"], a["x"], rtol=1e-9, atol=1e-12 * (1 + np.abs(a["x"]).max()))


def _worker(rank, world, port, kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import cuda_mpi_parallel_amd as mcg
    from cuda_mpi_parallel_amd.parallel.cpu_ref import cpu_cg_distributed, gather_x

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = cpu_cg_distributed(mcg.make_problem("randspd", **kw), maxit=2000, tol=1e-7)
        x = gather_x(out)
        if rank == 0:
            q.put((out["iterations"], out["converged"], x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_all_gather_path_matches_single_process(mcg, C, world):
    """world_size processes exchanging ghosts with dist.all_gather (the ncclAllGather plan)."""
    ref = C.cpu_cg(mcg.make_problem("randspd", **WIDE).native(), C.CgOptions(maxit=2000, tol=1e-7))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, WIDE, q)) for r in range(world)]
    for p in procs:
        p.start()
    its, conv, x = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert abs(its - ref["iterations"]) <= 1 and conv == ref["converged"]
    np.testing.assert_allclose(x, ref["x"], rtol=1e-7, atol=1e-9 * (1 + np.abs(ref["x"]).max()))
