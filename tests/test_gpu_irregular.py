"""GPU irregular-sparsity path (BASELINE.json config 5): the materialized-p split pass
(csrc/gpu/cg_split.hip) and the all-gather ghost layout, on one GPU and as P in-process ranks
(LocalComm; the RCCL all-gather itself runs in tests/test_gpu_rccl.py when >= 2 GPUs are visible).

Anchor: the reference's generic CSR SpMV (CUDACG.cu:213-216, 288) must handle any sparsity.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WIDE = dict(rows=20000, band=24, density=0.5, spread=20000)


def _cpu(mcg, spec, maxit=2000, tol=1e-7):
    C = mcg.native()
    return C.cpu_cg(spec.native(), C.CgOptions(maxit=maxit, tol=tol))


@pytest.mark.parametrize("fmt", ["csr", "sell", "sell16"])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=96)), ("randspd", dict(rows=20000, band=40, density=0.25)),
                                         ("randspd", WIDE)])
def test_split_pass_matches_cpu(mcg, fmt, problem, kw):
    spec = mcg.make_problem(problem, **kw)
    cpu = _cpu(mcg, spec)
    s = mcg.CGSolver(spec, format=fmt, recurrence=1, pmat=1, check_every=8)
    assert s.info["pmat"]
    out = s.solve()
    assert abs(out["iterations"] - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    assert out["converged"] == cpu["converged"]
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())
    assert s.true_residual_norm() < 1e-6


def test_split_pass_auto_for_wide_rows_and_same_recurrence_as_fused(mcg):
    spec = mcg.make_problem("randspd", rows=20000, band=64, density=0.5, spread=20000)
    a = mcg.CGSolver(spec, format="sell", recurrence=1, check_every=8)
    assert a.info["pmat"]  # >= 32 nonzeros per row and no LDS window: the split pass
    b = mcg.CGSolver(spec, format="sell", recurrence=1, pmat=0, check_every=8)
    assert not b.info["pmat"]
    ra, rb = a.solve(), b.solve()
    assert abs(ra["iterations"] - rb["iterations"]) <= 1  # same scalars, different sum blocking
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("fused", [-1, 0])
def test_split_pass_graph_equals_eager_bitwise(mcg, fused):
    spec = mcg.make_problem("randspd", **WIDE)
    outs = [mcg.CGSolver(spec, format="sell", recurrence=1, pmat=1, use_graph=g, fused_reduce=fused,
                         check_every=8).solve() for g in (True, False)]
    assert outs[0]["iterations"] == outs[1]["iterations"] and outs[0]["rnorm"] == outs[1]["rnorm"]
    np.testing.assert_array_equal(outs[0]["x_local"], outs[1]["x_local"])


def test_split_pass_fixed_iterations_track_fused(mcg):
    spec = mcg.make_problem("poisson2d", n=256, rhs="random")
    r = []
    for pm in (1, 0):
        s = mcg.CGSolver(spec, format="sell", recurrence=1, pmat=pm, tol=-1.0, maxit=300)
        r.append(s.solve())
    assert r[0]["iterations"] == r[1]["iterations"] == 300
    assert abs(r[0]["rnorm"] - r[1]["rnorm"]) <= 1e-10 * r[1]["rnorm"]


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_local_ranks_all_gather_layout(mcg, world):
    """P ranks on the wide matrix: all-gather layout + split pass, every rank latched together,
    x equal to the CPU oracle (a reduced-rows rehearsal of config 5)."""
    spec = mcg.make_problem("randspd", **WIDE)
    C = mcg.native()
    cpu = _cpu(mcg, spec)
    o = C.CgOptions(format="sell", recurrence=1, check_every=4)
    out = C.run_local_ranks(spec.native(), o, world, 0, True)
    its = {r["iterations"] for r in out["ranks"]}
    assert len(its) == 1
    assert abs(its.pop() - cpu["iterations"]) <= 1
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-8, atol=1e-10 * np.abs(cpu["x"]).max())
    assert all(r["true_rnorm"] < 1e-6 for r in out["ranks"])


def test_local_ranks_p8_agrees_with_p1_fixed_iterations(mcg):
    """Config-5 rehearsal: 8 ranks vs 1 over 12 fixed iterations on the wide matrix (strictly
    diagonally dominant: ~0.45x residual per iteration, so 12 keep the residual far above rounding)."""
    spec = mcg.make_problem("randspd", rows=40000, band=48, density=0.5, spread=40000)
    C = mcg.native()
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, format="sell", recurrence=1)
    one = C.run_local_ranks(spec.native(), o, 1, 12, True)
    eight = C.run_local_ranks(spec.native(), o, 8, 12, True)
    r1, r8 = one["ranks"][0]["rnorm"], eight["ranks"][0]["rnorm"]
    assert abs(r1 - r8) <= 1e-11 * r1
    np.testing.assert_allclose(eight["x"], one["x"], rtol=1e-12, atol=1e-14 * np.abs(one["x"]).max())


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("overlap", [True, False])
def test_local_ranks_split_pass_window_halo(mcg, world, overlap):
    """The split pass on a stencil with the column-window halo (p only), interior || halo."""
    spec = mcg.make_problem("poisson2d", n=64)
    C = mcg.native()
    cpu = _cpu(mcg, spec)
    o = C.CgOptions(format="sell16", recurrence=1, overlap=overlap, check_every=4)
    o.pmat = 1
    out = C.run_local_ranks(spec.native(), o, world, 0, True)
    its = {r["iterations"] for r in out["ranks"]}
    assert len(its) == 1 and abs(its.pop() - cpu["iterations"]) <= 2
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())


DENSE_WIDE = dict(rows=30000, band=64, density=1.0, spread=30000)


def test_aligned_sell_auto_and_same_row_sums(mcg):
    """SELL-64/aligned (one offset per slot, values only) stores the entries of SELL-64 in the same
    order plus zeros: the same recurrence, the CPU oracle's x, fewer matrix bytes per nonzero."""
    spec = mcg.make_problem("randspd", **DENSE_WIDE)
    a = mcg.CGSolver(spec, format="sell", recurrence=1, check_every=8)
    b = mcg.CGSolver(spec, format="sell", recurrence=1, check_every=8, sell_aligned=0)
    assert a.info["format"] == "sell64-aligned" and a.info["pmat"]
    assert b.info["format"] == "sell64"
    ra, rb = a.solve(), b.solve()
    assert ra["iterations"] == rb["iterations"]
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-13, atol=1e-15)
    cpu = _cpu(mcg, spec)
    np.testing.assert_allclose(ra["x_local"], cpu["x"], rtol=1e-8, atol=1e-10 * np.abs(cpu["x"]).max())
    assert a.true_residual_norm() < 1e-6


@pytest.mark.parametrize("world", [2, 4, 8])
def test_aligned_sell_local_ranks_all_gather(mcg, world):
    spec = mcg.make_problem("randspd", **DENSE_WIDE)
    C = mcg.native()
    cpu = _cpu(mcg, spec)
    o = C.CgOptions(format="sell", recurrence=1, check_every=4)
    out = C.run_local_ranks(spec.native(), o, world, 0, True)
    assert len({r["iterations"] for r in out["ranks"]}) == 1
    assert abs(out["ranks"][0]["iterations"] - cpu["iterations"]) <= 1
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-8, atol=1e-10 * np.abs(cpu["x"]).max())
    assert all(r["true_rnorm"] < 1e-6 for r in out["ranks"])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_all_gather_overlap_halves_match(mcg, world):
    """SELL-64/aligned on the all-gather layout: the own-block slots are summed while the all-gather
    of p is in flight, the rest after it (ag_overlap).  Same iterations and x as the one-pass SpMV
    and the CPU oracle; about 1/P of the slots are own-block for a matrix spread over all rows."""
    spec = mcg.make_problem("randspd", **DENSE_WIDE)
    C = mcg.native()
    cpu = _cpu(mcg, spec)
    outs = []
    for ag in (1, 0):
        o = C.CgOptions(format="sell", recurrence=1, check_every=4)
        o.ag_overlap = ag
        outs.append(C.run_local_ranks(spec.native(), o, world, 0, True))
    on, off = outs
    assert all(r["ag_overlap"] for r in on["ranks"]) and not any(r["ag_overlap"] for r in off["ranks"])
    frac = np.mean([r["ag_local_frac"] for r in on["ranks"]])
    assert 0.3 / world < frac < 2.0 / world
    assert len({r["iterations"] for r in on["ranks"]}) == 1
    assert abs(on["ranks"][0]["iterations"] - off["ranks"][0]["iterations"]) <= 1
    np.testing.assert_allclose(on["x"], off["x"], rtol=1e-10, atol=1e-12 * np.abs(off["x"]).max())
    np.testing.assert_allclose(on["x"], cpu["x"], rtol=1e-8, atol=1e-10 * np.abs(cpu["x"]).max())
    assert all(r["true_rnorm"] < 1e-6 for r in on["ranks"])


def test_all_gather_overlap_phase_profile(mcg):
    """phase_profile of the split pass with the halves: both SpMV halves are timed."""
    spec = mcg.make_problem("randspd", **DENSE_WIDE)
    C = mcg.native()
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, format="sell", recurrence=1)
    out = C.run_local_ranks(spec.native(), o, 4, 8, False, 4)
    ph = out["ranks"][0]["phases"]
    assert ph["spmv_local"] > 0 and ph["spmv"] > 0 and ph["halo"] >= 0


def test_null_comm_rank_share_takes_the_split_pass(mcg):
    """Per-rank timing rehearsal (NullComm) of the wide family: the setup-time agreement on the pass
    form takes the rank's own choice, so rank 3 of 8 runs aligned SELL, the split pass and the
    all-gather halves like a real 8-rank job."""
    spec = mcg.make_problem("randspd", **DENSE_WIDE)
    C = mcg.native()
    comm = C.NullComm(3, 8)
    s = C.Solver(spec.native(), C.CgOptions(format="sell", recurrence=1), 3, 8, comm)
    s.setup()
    info = s.info
    assert info["pmat"] and info["allgather"] and info["ag_overlap"] and info["format"] == "sell64-aligned"
    s.reset()
    s.run_iterations(6)
    s.synchronize()


# ---- scrambled random SPD (P^T A P: genuinely irregular) on L2-segment COO tiles ----
SCR = dict(rows=60000, band=24, density=0.5, scramble=1)


@pytest.mark.parametrize("seg", [19, 18, 12])
def test_tiles_scrambled_matches_cpu(mcg, seg):
    """The scrambled family takes the tiles SpMV by default; seg = 12 cuts p into 15 segments of 4096
    doubles (many tiles per row block, each segment step paced on the group's step flags); the solve
    matches the CPU oracle and ||b - A x||."""
    spec = mcg.make_problem("randspd", **SCR)
    cpu = _cpu(mcg, spec)
    s = mcg.CGSolver(spec, format="sellc8", recurrence=-1, check_every=8, tile_seg_log2=seg)
    assert s.info["tiles"] and s.info["pmat"] and s.info["format"] == "tiles"
    assert s.info["tile_segments"] == (1 if seg >= 18 else 15)
    out = s.solve()
    assert out["converged"] and abs(out["iterations"] - cpu["iterations"]) <= 1
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-8, atol=1e-10 * np.abs(cpu["x"]).max())
    assert s.true_residual_norm() < 1e-6


def test_tiles_same_recurrence_as_sell_split_and_deterministic(mcg):
    """Tiles vs the SELL split pass: the same scalars and vectors up to the rounding of the row sums
    (fixed iterations); two tile solvers built separately agree bit for bit (deterministic fill and
    in-order LDS sums), and a graph solve equals an eager one."""
    spec = mcg.make_problem("randspd", **SCR)
    kw = dict(format="sell", recurrence=1, tol=-1.0, maxit=40, tile_seg_log2=12)
    a = mcg.CGSolver(spec, tiles=1, **kw).solve()
    b = mcg.CGSolver(spec, tiles=0, pmat=1, **kw).solve()
    assert a["iterations"] == b["iterations"] == 40
    assert abs(a["rnorm"] - b["rnorm"]) <= 1e-10 * b["rnorm"]
    np.testing.assert_allclose(a["x_local"], b["x_local"], rtol=1e-12, atol=1e-14 * np.abs(b["x_local"]).max())
    c = mcg.CGSolver(spec, tiles=1, use_graph=False, **kw).solve()
    assert c["rnorm"] == a["rnorm"]
    np.testing.assert_array_equal(c["x_local"], a["x_local"])


def test_tiles_lane_depth_bitwise_and_chosen_by_tile_size(mcg, monkeypatch):
    """8 or 10 entries per lane in flight (kern::tiles_tu, MCG_TILES_TU overrides it): every row's
    adds run in ascending entry order either way, so the solves are bitwise equal; the default picks
    the depth whose batches of 64 x TU entries the mean tile fills better."""
    spec = mcg.make_problem("randspd", **SCR)
    kw = dict(format="sell", recurrence=1, tol=-1.0, maxit=30, tile_seg_log2=12, tiles=1)
    out = {}
    for tu in (8, 10):
        monkeypatch.setenv("MCG_TILES_TU", str(tu))
        s = mcg.CGSolver(spec, **kw)
        assert s.info["tiles"] and s.info["tiles_tu"] == tu
        out[tu] = s.solve()
    assert out[8]["rnorm"] == out[10]["rnorm"]
    np.testing.assert_array_equal(out[8]["x_local"], out[10]["x_local"])
    monkeypatch.delenv("MCG_TILES_TU")
    s = mcg.CGSolver(spec, **kw)
    m = s.info["nnz_local"] / (s.info["tile_segments"] * -(-s.info["n_local"] // 1024))

    def fill(tu):
        b = 64 * tu
        return m / (-(-m // b) * b)

    assert s.info["tiles_tu"] == (10 if fill(10) > fill(8) else 8)


def test_tiles_several_rounds_of_row_blocks(mcg):
    """More row blocks than waves (blocks_per_cu = 1: 1024 waves, 1.2 M rows = 1172 blocks): the
    waves take a second round of blocks; the same row sums as the full grid (only the dot products'
    block partials group differently)."""
    spec = mcg.make_problem("randspd", rows=1200000, band=4, density=0.5, scramble=1)
    kw = dict(format="sell", recurrence=1, tol=-1.0, maxit=12, tile_seg_log2=16)
    a = mcg.CGSolver(spec, blocks_per_cu=1, **kw)
    b = mcg.CGSolver(spec, **kw)
    assert a.info["tiles"] and a.info["grid_a"] < b.info["grid_a"]
    ra, rb = a.solve(), b.solve()
    assert abs(ra["rnorm"] - rb["rnorm"]) <= 1e-13 * rb["rnorm"]
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-13, atol=1e-15 * np.abs(rb["x_local"]).max())
    assert abs(a.true_residual_norm() - ra["rnorm"]) <= 1e-9 * ra["rnorm"]


def test_tiles_user_matrix_scattered(mcg):
    """A user CSR with scattered columns (random sparsity, strictly diagonally dominant) on the tiles
    SpMV (forced at P = 1; auto on the all-gather layout) matches the CPU reference solve."""
    import scipy.sparse as sp

    n = 20000
    rng = np.random.default_rng(3)
    rows = np.repeat(np.arange(n), 6)  # 6 random entries a row (sp.random would enumerate n^2 candidates)
    B = sp.csr_matrix((rng.random(6 * n), (rows, rng.integers(0, n, 6 * n))), shape=(n, n))
    B = B + B.T
    A = B + sp.diags(np.asarray(abs(B).sum(axis=1)).ravel() + 1.0)
    perm = rng.permutation(n)
    A = A[perm][:, perm].tocsr()
    b = rng.random(n)
    prob = mcg.csr_problem(A, b=b)
    s = mcg.CGSolver(prob, format="sell", recurrence=1, tiles=1, tol=1e-10, tile_seg_log2=12)
    assert s.info["tiles"]
    out = s.solve()
    cpu = _cpu(mcg, prob, tol=1e-10)
    assert out["converged"] and abs(out["iterations"] - cpu["iterations"]) <= 1
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-8, atol=1e-10)


def test_tiles_auto_for_scattered_user_matrix_at_one_rank(mcg):
    """P = 1, no all-gather layout: a user CSR with >= 1/4 of its entries beyond 2^16 columns of
    their row (HostMatrix.far_entries) takes the tiles by itself; a banded one keeps SELL.  The two
    SpMVs agree over 30 fixed iterations."""
    import scipy.sparse as sp

    n = 200000
    rng = np.random.default_rng(5)
    # 8 random entries a row, built from index draws (sp.random would enumerate n^2 candidates)
    rows = np.repeat(np.arange(n), 8)
    B = sp.csr_matrix((rng.random(8 * n), (rows, rng.integers(0, n, 8 * n))), shape=(n, n))
    B = B + B.T
    A = (B + sp.diags(np.asarray(abs(B).sum(axis=1)).ravel() + 1.0)).tocsr()
    b = rng.random(n)
    prob = mcg.csr_problem(A, b=b)
    assert 4 * prob.matrix.far_entries >= A.nnz
    kw = dict(format="sell", recurrence=1, tol=-1.0, maxit=30)
    t = mcg.CGSolver(prob, **kw)
    assert t.info["tiles"]
    plain = mcg.CGSolver(prob, tiles=0, **kw)
    assert not plain.info["tiles"]
    rt, rp = t.solve(), plain.solve()
    assert rt["iterations"] == rp["iterations"] == 30
    assert abs(rt["rnorm"] - rp["rnorm"]) <= 1e-10 * rp["rnorm"]
    T = sp.diags([-1.0, 2.5, -1.0], [-1, 0, 1], shape=(n, n)).tocsr()
    banded = mcg.csr_problem(T, b=b)
    assert banded.matrix.far_entries == 0
    assert not mcg.CGSolver(banded, **kw).info["tiles"]


def test_tiles_local_ranks_p8_agrees_with_p1(mcg):
    """Config-5 rehearsal on the scrambled matrix: 8 LocalComm ranks (all-gather layout, tiles on
    every rank) vs 1 rank over 12 fixed iterations agree to <= 1e-13."""
    spec = mcg.make_problem("randspd", rows=80000, band=32, density=0.5, scramble=1)
    C = mcg.native()
    o = C.CgOptions(tol=-1.0, maxit=1 << 30, format="sell", recurrence=1)
    o.tile_seg_log2 = 13
    one = C.run_local_ranks(spec.native(), o, 1, 12, True)
    eight = C.run_local_ranks(spec.native(), o, 8, 12, True)
    r1, r8 = one["ranks"][0]["rnorm"], eight["ranks"][0]["rnorm"]
    assert abs(r1 - r8) <= 1e-13 * r1
    np.testing.assert_allclose(eight["x"], one["x"], rtol=1e-13, atol=1e-15 * np.abs(one["x"]).max())
    assert all(abs(r["true_rnorm"] - r8) <= 1e-9 * r8 for r in eight["ranks"])


def test_tiles_row_colliding_batches_run_to_run_bitwise(mcg):
    """lanes of one ds_add_f64 batch may target the same row's LDS sum.  Ten dense
    rows with 300 entries each inside one 4096-column segment force it (every 64-entry batch of their
    tile holds at most 10 distinct rows).  The order of same-address lanes inside one LDS atomic is a
    hardware behaviour, not an architectural guarantee; on MI355X it is observed fixed: repeated
    solves, graph and eager, are bit for bit equal (cg_tiles.hip documents exactly this)."""
    import scipy.sparse as sp

    n = 20000
    rng = np.random.default_rng(11)
    rows = [np.repeat(np.arange(n), 4), np.repeat(np.arange(10), 300)]
    cols = [rng.integers(0, n, 4 * n), rng.integers(0, 4096, 3000)]
    B = sp.csr_matrix((rng.random(4 * n + 3000), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    B = B + B.T
    A = (B + sp.diags(np.asarray(abs(B).sum(axis=1)).ravel() + 1.0)).tocsr()
    assert A[:10, :4096].getnnz(axis=1).min() > 64
    prob = mcg.csr_problem(A, b=rng.random(n))
    outs = []
    for graph in (True, True, False):
        s = mcg.CGSolver(prob, format="sell", recurrence=1, tiles=1, tol=-1.0, maxit=25, tile_seg_log2=12,
                         use_graph=graph)
        assert s.info["tiles"]
        outs.append(s.solve())
    for o in outs[1:]:
        assert o["rnorm"] == outs[0]["rnorm"]
        np.testing.assert_array_equal(o["x_local"], outs[0]["x_local"])


@pytest.mark.parametrize("world", [2, 8])
def test_tiles_all_gather_overlap_halves_match(mcg, world):
    """Tiles on the all-gather layout (scrambled family): the column segments inside a rank's own
    block of p are swept while the all-gather of p_k is in flight (part 1, partial row sums stored in
    Ap), the other segments after it (part 2).  Against the one-launch sweep: same iterations, x to
    rounding (the two halves add a row's products in another order), the CPU oracle, and ~1/P of
    the entries in the own segments."""
    spec = mcg.make_problem("randspd", rows=80000, band=32, density=0.5, scramble=1)
    C = mcg.native()
    cpu = _cpu(mcg, spec)
    outs = []
    for ag in (1, 0):
        o = C.CgOptions(format="sell", recurrence=1, check_every=4)
        o.tile_seg_log2 = 10
        o.ag_overlap = ag
        outs.append(C.run_local_ranks(spec.native(), o, world, 0, True))
    on, off = outs
    assert all(r["ag_overlap"] for r in on["ranks"]) and not any(r["ag_overlap"] for r in off["ranks"])
    frac = np.mean([r["ag_local_frac"] for r in on["ranks"]])
    assert 0.5 / world < frac < 1.5 / world
    assert len({r["iterations"] for r in on["ranks"]}) == 1
    assert abs(on["ranks"][0]["iterations"] - off["ranks"][0]["iterations"]) <= 1
    np.testing.assert_allclose(on["x"], off["x"], rtol=1e-10, atol=1e-12 * np.abs(off["x"]).max())
    np.testing.assert_allclose(on["x"], cpu["x"], rtol=1e-8, atol=1e-10 * np.abs(cpu["x"]).max())
    assert all(r["true_rnorm"] < 1e-6 for r in on["ranks"])


@pytest.mark.parametrize("ww", [8, 16])
def test_tiles_wide_workgroups_same_row_sums(mcg, ww):
    """PassForm::tile_waves = 16 / 8 (one 1024- or two 512-thread workgroups per CU, the pacing barrier
    over waves of one age): every row's sum is added in the same order as with four 4-wave workgroups
    (its wave owns it), so the iterates agree to the rounding of the dot products' block partials
    (grouped over 16 / 8 waves instead of 4); graph = eager bit for bit and the true residual tracks."""
    spec = mcg.make_problem("randspd", **SCR)
    kw = dict(format="sell", recurrence=1, tol=-1.0, maxit=40, tile_seg_log2=12, tiles=1)
    a = mcg.CGSolver(spec, **kw).solve()
    s = mcg.CGSolver(spec, tile_waves=ww, **kw)
    assert s.info["tiles"]
    b = s.solve()
    assert a["iterations"] == b["iterations"] == 40
    assert abs(a["rnorm"] - b["rnorm"]) <= 1e-12 * a["rnorm"]
    np.testing.assert_allclose(b["x_local"], a["x_local"], rtol=1e-12, atol=1e-14 * np.abs(a["x_local"]).max())
    c = mcg.CGSolver(spec, tile_waves=ww, use_graph=False, **kw).solve()
    assert c["rnorm"] == b["rnorm"]
    np.testing.assert_array_equal(c["x_local"], b["x_local"])
    tr = s.true_residual_norm()
    assert abs(tr - b["rnorm"]) <= 1e-8 * tr
