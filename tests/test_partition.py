"""1-D row partition and halo plan (csrc/host/partition.cpp) — the data structures the
RCCL halo exchange is driven by.  Property tests over problems and rank counts."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st


def _layouts(mcg, spec, world):
    return [mcg.parallel.layout(spec, world, r) for r in range(world)]


@settings(max_examples=60, deadline=None)
@given(problem=st.sampled_from(["poisson2d", "poisson3d", "randspd", "demo"]), n=st.integers(2, 24),
       world=st.integers(1, 9))
def test_plan_properties(mcg, problem, n, world):
    kw = {"poisson2d": dict(n=n), "poisson3d": dict(n=max(2, n // 3)),
          "randspd": dict(rows=n * 37, band=max(1, n // 2), density=0.4), "demo": {}}[problem]
    spec = mcg.make_problem(problem, **kw)
    Ls = _layouts(mcg, spec, world)
    # partition covers [0, n) contiguously
    assert Ls[0].row_begin == 0 and Ls[-1].row_end == spec.n_rows
    for a, b in zip(Ls, Ls[1:]):
        assert a.row_end == b.row_begin
    for L in Ls:
        assert L.own_off % 8 == 0 and L.ext_len >= L.own_off + L.n_local
        assert 0 <= L.interior_begin <= L.interior_end <= L.n_local
        # sends of r to q == recvs of q from r, same ranges in the same order (RCCL matching rule)
        for q in range(world):
            s = [(g, c) for (p, g, c) in L.sends if p == q]
            r = [(g, c) for (p, g, c) in Ls[q].recvs if p == L.rank]
            assert s == r
        # every column of every owned row is owned or arrives by exactly one recv
        cover = np.zeros(spec.n_rows, dtype=int)
        for (_, g, c) in L.recvs:
            cover[g:g + c] += 1
        assert cover.max(initial=0) <= 1
        nat = spec.native()
        for i in range(L.row_begin, L.row_end):
            cols, _ = nat.row(i)
            local = i - L.row_begin
            interior = L.interior_begin <= local < L.interior_end
            for c in cols:
                owned = L.row_begin <= c < L.row_end
                assert owned or cover[c] == 1
                if interior:
                    assert owned
                assert 0 <= L.ext_index(c) < L.ext_len


def test_stencil_partition_is_line_aligned(mcg):
    spec = mcg.make_problem("poisson2d", n=16384)
    offs = mcg.parallel.partition_rows(spec, 8)
    assert all(o % 16384 == 0 for o in offs)
    L = mcg.parallel.layout(spec, 8, 3)
    # neighbours only, one grid line (N rows = 128 KiB of doubles) each way
    assert sorted(p for p, _, _ in L.recvs) == [2, 4]
    assert all(c == 16384 for _, _, c in L.recvs + L.sends)
    assert L.interior_end - L.interior_begin == L.n_local - 2 * 16384


def test_3d_partition_plane_aligned(mcg):
    spec = mcg.make_problem("poisson3d", n=512)
    offs = mcg.parallel.partition_rows(spec, 8)
    assert all(o % (512 * 512) == 0 for o in offs)
    L = mcg.parallel.layout(spec, 8, 0)
    assert L.recvs == ((1, 64 * 512 * 512, 512 * 512),)


def test_more_ranks_than_lines_falls_back_to_rows(mcg):
    spec = mcg.make_problem("poisson2d", n=4)  # 16 rows, 4 lines
    offs = mcg.parallel.partition_rows(spec, 8)
    assert offs[0] == 0 and offs[-1] == 16 and all(b - a == 2 for a, b in zip(offs, offs[1:]))


def test_partition_by_weight(C):
    prefix = np.concatenate([[0], np.cumsum([1] * 50 + [100] * 10)]).tolist()
    offs = C.partition_by_weight(prefix, 4)
    w = [prefix[b] - prefix[a] for a, b in zip(offs, offs[1:])]
    assert offs[0] == 0 and offs[-1] == 60
    assert max(w) <= 2 * (prefix[-1] / 4)


def _spmv_rows(rowptr, cols, vals, xe):
    """y_i = sum_j a_ij x_j in stored entry order (sequential fp64, like every engine's row sum)."""
    y = np.zeros(len(rowptr) - 1)
    for i in range(len(rowptr) - 1):
        s = 0.0
        for k in range(rowptr[i], rowptr[i + 1]):
            s = s + vals[k] * xe[cols[k]]
        y[i] = s
    return y


@pytest.mark.parametrize("problem,kw,world", [("poisson2d", dict(n=12), 3), ("poisson3d", dict(n=5), 4),
                                               ("randspd", dict(rows=300, band=20, density=0.5), 5),
                                               # band >= rows: every rank needs every other rank's rows
                                               # (the dense-halo / full-replica case)
                                               ("randspd", dict(rows=200, band=200, density=0.05), 3)])
def test_partitioned_spmv_with_ghost_copies_is_bitwise_global(mcg, problem, kw, world):
    """Per-rank CSR (ext-local columns) + ghost rows copied along the halo plan reproduces the
    global SpMV bit for bit (SURVEY.md §4.3 'simulated distribution')."""
    spec = mcg.make_problem(problem, **kw)
    C = mcg.native()
    n = spec.n_rows
    x = np.random.default_rng(7).standard_normal(n)
    rp, cols, vals = C.host_csr(spec.native(), 1, 0)
    y_global = _spmv_rows(rp, cols, vals, x)
    Ls = _layouts(mcg, spec, world)
    y = np.zeros(n)
    for L in Ls:
        xe = np.full(L.ext_len, np.nan)  # anything not delivered by the plan poisons the result
        xe[L.own_off:L.own_off + L.n_local] = x[L.row_begin:L.row_end]
        for (_, g, c) in L.recvs:
            xe[L.ext_index(g):L.ext_index(g) + c] = x[g:g + c]
        rp_l, cols_l, vals_l = C.host_csr(spec.native(), world, L.rank)
        y[L.row_begin:L.row_end] = _spmv_rows(rp_l, cols_l, vals_l, xe)
    np.testing.assert_array_equal(y, y_global)
    for L in Ls:
        assert 0 <= L.interior_begin <= L.interior_end <= L.n_local
    if kw.get("band", 0) >= n:
        assert any(sum(c for (_, _, c) in L.recvs) == n - L.n_local for L in Ls)  # full replica
