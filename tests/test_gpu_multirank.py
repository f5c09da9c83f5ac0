"""Multi-rank solver on one GPU: P ranks as threads with the in-process LocalComm.

RCCL refuses several ranks on one device, so this harness is how the distributed
path (partition, halo plan, ghost layout, interior/boundary split + side-stream
overlap, collective placement, latch agreement) is checked on a single MI355X with
the same kernels the RCCL path launches.  The RCCL calls themselves are covered by
the 1-rank force_comm test and by the driver's multi-GPU runs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _opts(mcg, **kw):
    return mcg.native().CgOptions(**kw)


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("recurrence", [0, 1])
@pytest.mark.parametrize("fmt,overlap", [("csr", True), ("sell16", True), ("sell", False), ("sellc8", True)])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=64)), ("poisson3d", dict(n=16)),
                                         ("randspd", dict(rows=6000, band=30, density=0.3))])
def test_local_ranks_match_cpu(mcg, world, recurrence, fmt, overlap, problem, kw):
    spec = mcg.make_problem(problem, **kw)
    C = mcg.native()
    cpu = C.cpu_cg(spec.native(), C.CgOptions(maxit=2000, tol=1e-7))
    out = C.run_local_ranks(spec.native(), _opts(mcg, format=fmt, overlap=overlap, recurrence=recurrence,
                                                 check_every=4), world, 0, True)
    its = {r["iterations"] for r in out["ranks"]}
    assert len(its) == 1, its  # every rank latched at the same iteration
    it = its.pop()
    assert abs(it - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    assert all(r["converged"] == cpu["converged"] for r in out["ranks"])
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())
    assert all(r["true_rnorm"] < 1e-6 for r in out["ranks"])


@pytest.mark.parametrize("recurrence", [0, 1])
def test_local_ranks_fixed_iterations_agree_with_single_rank(mcg, recurrence):
    """Same fixed number of iterations at P = 1 and P = 4: residual histories agree to rounding."""
    spec = mcg.make_problem("poisson2d", n=256)
    C = mcg.native()
    o = _opts(mcg, tol=-1.0, maxit=1 << 30, format="sell16", recurrence=recurrence)
    one = C.run_local_ranks(spec.native(), o, 1, 40, True)
    four = C.run_local_ranks(spec.native(), o, 4, 40, True)
    r1 = one["ranks"][0]["rnorm"]
    r4 = four["ranks"][0]["rnorm"]
    assert abs(r1 - r4) <= 1e-9 * r1
    np.testing.assert_allclose(four["x"], one["x"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("world", [2, 3])
def test_local_ranks_interleaved_halo_bitwise(mcg, world):
    """Halo exchange of the 16-B {r, Ap} pairs (width-2 messages) vs split vectors."""
    spec = mcg.make_problem("poisson3d", n=16)
    C = mcg.native()
    outs = []
    for il in (1, 0):
        o = _opts(mcg, format="sell16", recurrence=1, check_every=4)
        o.interleave = il
        outs.append(C.run_local_ranks(spec.native(), o, world, 0, True))
    assert [r["iterations"] for r in outs[0]["ranks"]] == [r["iterations"] for r in outs[1]["ranks"]]
    np.testing.assert_array_equal(outs[0]["x"], outs[1]["x"])


@pytest.mark.parametrize("recurrence,fmt", [(0, "csr"), (1, "sellc8"), (1, "sell16")])
def test_local_ranks_dense_halo_full_replica(mcg, recurrence, fmt):
    """band >= rows: each rank gathers every other rank's rows (all-gather-shaped halo)."""
    spec = mcg.make_problem("randspd", rows=3000, band=3000, density=0.01)
    C = mcg.native()
    cpu = C.cpu_cg(spec.native(), C.CgOptions(maxit=2000, tol=1e-7))
    out = C.run_local_ranks(spec.native(), _opts(mcg, format=fmt, recurrence=recurrence, check_every=4), 3, 0, True)
    assert abs(out["ranks"][0]["iterations"] - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())
    assert all(r["true_rnorm"] < 1e-6 for r in out["ranks"])


@pytest.mark.parametrize("world", [2, 3])
def test_local_ranks_window_pass_bitwise(mcg, world):
    """Windowed pass with interior/boundary split + halo overlap vs the plain pass (same row sums;
    the dot-product partials are blocked differently, so agreement is to rounding)."""
    spec = mcg.make_problem("randspd", rows=9000, band=50, density=0.7)
    C = mcg.native()
    outs = []
    for w in (1, 0):
        o = _opts(mcg, format="sell16", recurrence=1, check_every=4)
        o.window = w
        outs.append(C.run_local_ranks(spec.native(), o, world, 0, True))
    assert [r["iterations"] for r in outs[0]["ranks"]] == [r["iterations"] for r in outs[1]["ranks"]]
    np.testing.assert_allclose(outs[0]["x"], outs[1]["x"], rtol=1e-12, atol=1e-15)
    assert all(r["converged"] for r in outs[0]["ranks"])


@pytest.mark.parametrize("world", [2, 3])
def test_local_ranks_pipelined_pass_bitwise(mcg, world):
    spec = mcg.make_problem("poisson2d", n=200)
    C = mcg.native()
    outs = []
    for pp in (1, 0):
        o = _opts(mcg, format="sellc8", recurrence=1, check_every=4)
        o.pipeline = pp
        outs.append(C.run_local_ranks(spec.native(), o, world, 0, True))
    assert [r["iterations"] for r in outs[0]["ranks"]] == [r["iterations"] for r in outs[1]["ranks"]]
    np.testing.assert_array_equal(outs[0]["x"], outs[1]["x"])


def test_local_ranks_demo_more_ranks_than_rows_per_rank(mcg):
    """3x3 demo on 2 ranks (halo covers most of the matrix) still prints the golden x."""
    C = mcg.native()
    out = C.run_local_ranks(mcg.make_problem("demo").native(), _opts(mcg), 2, 0, False)
    assert "".join("%f\n" % v for v in out["x"]) == "0.500000\n0.750000\n1.000000\n"
    assert out["ranks"][0]["iterations"] == 3


@pytest.mark.parametrize("world", [2, 3])
def test_local_ranks_line_carry_interior(mcg, world):
    """Line-carry pass on the interior launch (boundary lines through the generic pass after the
    halo) across ranks vs the CPU reference."""
    spec = mcg.make_problem("poisson2d", n=192)
    C = mcg.native()
    cpu = C.cpu_cg(spec.native(), C.CgOptions(maxit=2000, tol=1e-7))
    o = _opts(mcg, format="sellc8", recurrence=1, check_every=4)
    o.carry = 1
    out = C.run_local_ranks(spec.native(), o, world, 0, True)
    assert all(r["carry"] for r in out["ranks"])
    its = {r["iterations"] for r in out["ranks"]}
    assert len(its) == 1, its
    assert abs(its.pop() - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())
    assert all(r["true_rnorm"] < 1e-6 for r in out["ranks"])


@pytest.mark.parametrize("world", [2, 4])
def test_local_ranks_plane_carry_interior(mcg, world):
    """3-D plane carry (the +-N rows gathered a plane ahead) on the interior planes of each rank,
    the two boundary planes through the generic pass after the halo, vs the same ranks without
    the carry pass (same row sums: agreement to rounding of the dot-product blocking)."""
    spec = mcg.make_problem("poisson3d", n=16)  # 16 planes of 256 rows: whole planes per rank
    C = mcg.native()
    outs = []
    for carry in (-1, 0):
        o = _opts(mcg, format="sellc8", recurrence=1, check_every=4)
        o.carry = carry
        outs.append(C.run_local_ranks(spec.native(), o, world, 0, True))
    assert all(r["carry"] for r in outs[0]["ranks"]) and not any(r["carry"] for r in outs[1]["ranks"])
    assert [r["iterations"] for r in outs[0]["ranks"]] == [r["iterations"] for r in outs[1]["ranks"]]
    np.testing.assert_allclose(outs[0]["x"], outs[1]["x"], rtol=1e-10, atol=1e-13)
    assert all(r["converged"] and r["true_rnorm"] < 1e-6 for r in outs[0]["ranks"])


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("problem,n", [("poisson2d", 256), ("poisson3d", 32), ("poisson3d", 64)])
@pytest.mark.parametrize("ar", [-1, 0])
def test_local_ranks_halo_ahead_matches_split(mcg, world, problem, n, ar):
    """halo_ahead (ghosts of iteration k+1 exchanged right after pass k, one full pass per
    iteration) against the interior || halo + boundary split and P = 1: same recurrence, so the
    residuals agree to rounding of the differently grouped partial sums."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    C = mcg.native()
    outs = {}
    for ha in (1, 0):
        o = _opts(mcg, tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1)
        o.halo_ahead = ha
        o.ap_recompute = ar  # auto: the 2-D carry recomputes Ap (ghost lines' Ap from the halo)
        outs[ha] = C.run_local_ranks(spec.native(), o, world, 60, True)
    one = C.run_local_ranks(spec.native(), _opts(mcg, tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1),
                            1, 60, True)
    r = one["ranks"][0]["rnorm"]
    for ha, out in outs.items():
        assert all(q["iterations"] == 60 for q in out["ranks"]), ha
        assert abs(out["ranks"][0]["rnorm"] - r) <= 1e-11 * r, ha
        np.testing.assert_allclose(out["x"], one["x"], rtol=1e-10, atol=1e-13)
        assert all(abs(q["true_rnorm"] - q["rnorm"]) <= 1e-8 * q["true_rnorm"] for q in out["ranks"])
    if problem == "poisson2d" or n % 64 == 0:  # the full pass of every rank is the line / plane carry
        assert all(q["carry"] for q in outs[1]["ranks"])
        assert all(q["ap_recompute"] == (ar != 0) for q in outs[1]["ranks"])
        assert not any(q["ap_recompute"] for q in outs[0]["ranks"])  # the split keeps the stored Ap


@pytest.mark.parametrize("problem,n", [("poisson2d", 512), ("poisson3d", 64)])
def test_null_comm_halo_ahead_graph_equals_eager(mcg, problem, n):
    """A P = 8 rank's share with collectives that move nothing (NullComm): the captured graphs
    (prefetch fork + join per iteration, the last one joined inside the graph) run exactly the
    eager iterations, bit for bit, with no capture fallback."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    C = mcg.native()
    xs, infos = [], []
    for graph in (True, False):
        o = C.CgOptions(tol=-1.0, maxit=1 << 30, check_every=1 << 30, format="sellc8", recurrence=1)
        o.use_graph = graph
        s = C.Solver(spec.native(), o, 3, 8, C.NullComm(3, 8))
        s.setup()
        s.reset()
        s.run_iterations(5)   # eager start, then graphs from an even k
        s.run_iterations(70)  # 32-iteration graphs + pair tail
        s.synchronize()
        s.finalize()
        xs.append(s.x_local())
        infos.append(dict(s.info, **s.result()))
    assert infos[0]["halo_ahead"] and infos[0]["graph_fallbacks"] == 0
    assert infos[0]["iterations"] == infos[1]["iterations"] == 75
    np.testing.assert_array_equal(xs[0], xs[1])


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=512)), ("poisson3d", dict(n=64))])
def test_local_ranks_default_serial_order_matches_single_rank(mcg, world, problem, kw):
    """The P > 1 default since r3 (`--comm single`: the collectives in one stream order, overlap
    off): the Ap-recomputing dia4 three-term carry over each rank's whole grid, the {Ap, p} halo
    before the pass.  Vs the CPU oracle, and vs P = 1 over 40 fixed iterations (<= 1e-12)."""
    spec = mcg.make_problem(problem, rhs="random", **kw)
    C = mcg.native()
    o = _opts(mcg, format="sellc8", recurrence=-1, check_every=4, overlap=False)
    out = C.run_local_ranks(spec.native(), o, world, 0, True)
    assert all(r["carry"] and r["ap_recompute"] for r in out["ranks"])
    its = {r["iterations"] for r in out["ranks"]}
    assert len(its) == 1, its
    cpu = C.cpu_cg(spec.native(), C.CgOptions(maxit=2000, tol=1e-7))
    assert abs(its.pop() - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())
    o = _opts(mcg, format="sellc8", recurrence=-1, tol=-1.0, maxit=1 << 30, overlap=False)
    one = C.run_local_ranks(spec.native(), o, 1, 40, True)
    many = C.run_local_ranks(spec.native(), o, world, 40, True)
    r1, rp = one["ranks"][0]["rnorm"], many["ranks"][0]["rnorm"]
    assert abs(r1 - rp) <= 1e-12 * r1
    np.testing.assert_allclose(many["x"], one["x"], rtol=1e-12, atol=1e-14 * np.abs(one["x"]).max())


@pytest.mark.parametrize("problem,n,world", [("poisson2d", 2048, 2), ("poisson2d", 2048, 4), ("poisson3d", 128, 2)])
def test_local_ranks_lean_runs_bitwise(mcg, problem, n, world):
    """With ghost lines (P > 1) the lean runs of the three-term dia4 carry take the runs clear of the
    rank's outer lines; every rank's x and the iteration count are bit for bit those of
    dia_uniform = 0 (the generic step for every run), on one grid (4 blocks per CU: the auto lean grids
    differ from the generic pass's, and the block partials' order with them)."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    C = mcg.native()
    outs = []
    for du in (-1, 0):
        o = _opts(mcg, tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1, check_every=8, blocks_per_cu=4)
        o.dia_uniform = du
        outs.append(C.run_local_ranks(spec.native(), o, world, 30, True))
    assert [r["rnorm"] for r in outs[0]["ranks"]] == [r["rnorm"] for r in outs[1]["ranks"]]
    np.testing.assert_array_equal(outs[0]["x"], outs[1]["x"])


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=4096)), ("poisson3d", dict(n=128)),
                                         ("poisson2d", dict(n=2048, coef=1)), ("poisson3d", dict(n=128, coef=1))])
def test_local_ranks_in_kernel_halo_bitwise(mcg, world, problem, kw):
    """the in-kernel halo (halo_pull).  From iteration 2 on the lean carries read
    their ghost lines / planes straight from the neighbours' rows (LocalComm: the other threads'
    buffers) and store their own first / last ones write-through, with no halo step -- bit for bit
    the serial path (halo exchanged before each pass) and the halo-ahead path, over 40 iterations."""
    spec = mcg.make_problem(problem, rhs="random", **kw)
    C = mcg.native()
    outs = {}
    for tag, hp, ov in (("pull", 1, False), ("serial", 0, False), ("ahead", 0, True), ("pull_ov", -1, True)):
        o = _opts(mcg, tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1, check_every=8, overlap=ov)
        o.halo_pull = hp
        o.probe_pick_halo = 1  # auto: the transport probe runs both arms, keeps the pull if it reproduced the exchange
        outs[tag] = C.run_local_ranks(spec.native(), o, world, 40, True)
        assert all(q["halo_pull"] == (hp != 0) for q in outs[tag]["ranks"]), (tag, outs[tag]["ranks"])
        assert all(q["probe_ran"] == (hp == -1) for q in outs[tag]["ranks"]), tag
        if hp == -1:
            assert all(q["probe_pull_bitwise"] and q["probe_pull_us"] > 0 and q["probe_xchg_us"] > 0
                       for q in outs[tag]["ranks"]), outs[tag]["ranks"]
        assert all(q["lean_only"] for q in outs[tag]["ranks"]), tag
    for tag in ("serial", "ahead", "pull_ov"):
        assert [q["rnorm"] for q in outs[tag]["ranks"]] == [q["rnorm"] for q in outs["pull"]["ranks"]], tag
        np.testing.assert_array_equal(outs[tag]["x"], outs["pull"]["x"])
    assert all(abs(q["true_rnorm"] - q["rnorm"]) <= 1e-8 * q["true_rnorm"] for q in outs["pull"]["ranks"])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_local_ranks_p3buf_bitwise(mcg, world):
    """Three p buffers at P > 1 (the ghost lines' / planes' p_{k-2} in the third buffer's ghost rows,
    pulled or exchanged): bit for bit the two-buffer lean pass, 2-D and 3-D, with the in-kernel halo
    and with the halo exchanged, over 40 iterations."""
    C = mcg.native()
    for prob, n, hp, coef in (("poisson2d", 4096, 1, 0), ("poisson2d", 4096, 0, 0), ("poisson3d", 128, 1, 0),
                              ("poisson3d", 128, 0, 0), ("poisson3d", 128, 1, 1), ("poisson2d", 2048, 1, 1)):
        spec = mcg.make_problem(prob, n=n, rhs="random", coef=coef)
        outs = {}
        for pb in (1, 0):
            o = _opts(mcg, tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1, check_every=8, overlap=False)
            o.halo_pull = hp
            o.p3buf = pb
            outs[pb] = C.run_local_ranks(spec.native(), o, world, 40, True)
        assert [q["rnorm"] for q in outs[1]["ranks"]] == [q["rnorm"] for q in outs[0]["ranks"]], (prob, hp)
        np.testing.assert_array_equal(outs[1]["x"], outs[0]["x"])


@pytest.mark.parametrize("problem,n", [("poisson2d", 2048), ("poisson3d", 64)])
def test_local_ranks_in_kernel_halo_converges(mcg, problem, n):
    """The in-kernel halo to convergence at P = 4 against the CPU oracle (the reference's recurrence)."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    C = mcg.native()
    o = _opts(mcg, format="sellc8", recurrence=-1, check_every=4)
    o.probe_pick_halo = 1  # (the probe's timing would pick either on threads sharing one GPU)
    out = C.run_local_ranks(spec.native(), o, 4, 0, True)
    assert all(q["halo_pull"] and q["probe_pull_bitwise"] for q in out["ranks"])
    its = {q["iterations"] for q in out["ranks"]}
    assert len(its) == 1, its
    cpu = C.cpu_cg(spec.native(), C.CgOptions(maxit=2000, tol=1e-7))
    assert abs(its.pop() - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    np.testing.assert_allclose(out["x"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())


@pytest.mark.parametrize("problem,n", [("poisson2d", 4096), ("poisson3d", 128)])
def test_null_comm_in_kernel_halo_graph_equals_eager(mcg, problem, n):
    """A P = 8 rank's share with the in-kernel halo forced on a NullComm (the rank's own first / last
    line stands in for the neighbours'): the 32-iteration graphs replay the eager pulled passes bit for
    bit, and a resumed count (graphs start only once pulling) keeps them equal."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    C = mcg.native()
    xs, infos = [], []
    for graph in (True, False):
        o = C.CgOptions(tol=-1.0, maxit=1 << 30, check_every=1 << 30, format="sellc8", recurrence=1)
        o.use_graph = graph
        o.halo_pull = 1
        s = C.Solver(spec.native(), o, 3, 8, C.NullComm(3, 8))
        s.setup()
        s.reset()
        s.run_iterations(5)
        s.run_iterations(70)
        s.synchronize()
        s.finalize()
        xs.append(s.x_local())
        infos.append(dict(s.info, **s.result()))
    assert infos[0]["halo_pull"] and infos[0]["graph_fallbacks"] == 0 and infos[0]["graphs"]
    assert infos[0]["iterations"] == infos[1]["iterations"] == 75
    np.testing.assert_array_equal(xs[0], xs[1])
