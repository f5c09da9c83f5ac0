"""GPU solver end-to-end: reference golden output, agreement with the CPU reference path."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_demo_golden(mcg):
    out = mcg.solve("demo")
    assert "".join("%f\n" % v for v in out["x_local"]) == "0.500000\n0.750000\n1.000000\n"
    assert out["iterations"] == 3 and out["converged"]
    assert out["rnorm"] < 1e-7


def test_cli_no_args_golden(mcg):
    p = subprocess.run([mcg.cli_path()], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout == "0.500000\n0.750000\n1.000000\nSuccess\n"


@pytest.mark.parametrize("fmt", ["csr", "sell", "sell16", "sellc8"])
@pytest.mark.parametrize("graph", [True, False])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=96)), ("poisson3d", dict(n=20)),
                                         ("randspd", dict(rows=20000, band=40, density=0.25))])
def test_matches_cpu_reference(mcg, fmt, graph, problem, kw):
    spec = mcg.make_problem(problem, **kw)
    cpu = mcg.native().cpu_cg(spec.native(), mcg.native().CgOptions(maxit=2000, tol=1e-7))
    s = mcg.CGSolver(spec, format=fmt, use_graph=graph, check_every=8)
    out = s.solve()
    # same recurrence, different summation order: iteration counts may differ by a step or two
    assert abs(out["iterations"] - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    assert out["converged"] == cpu["converged"]
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())
    tr = s.true_residual_norm()
    assert tr < 1e-6


@pytest.mark.parametrize("fmt", ["csr", "sell", "sell16", "sellc8"])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=96)), ("poisson3d", dict(n=20)),
                                         ("randspd", dict(rows=20000, band=40, density=0.25))])
def test_single_reduction_matches_cpu(mcg, fmt, problem, kw):
    spec = mcg.make_problem(problem, **kw)
    cpu = mcg.native().cpu_cg(spec.native(), mcg.native().CgOptions(maxit=2000, tol=1e-7))
    s = mcg.CGSolver(spec, format=fmt, recurrence=1, check_every=8)
    out = s.solve()
    assert abs(out["iterations"] - cpu["iterations"]) <= max(2, cpu["iterations"] // 100)
    assert out["converged"] == cpu["converged"]
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-6, atol=1e-6 * np.abs(cpu["x"]).max())
    assert s.true_residual_norm() < 1e-6


@pytest.mark.parametrize("fmt", ["sell", "sell16"])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=96)), ("randspd", dict(rows=20000, band=40, density=0.25))])
def test_interleaved_pairs_bitwise_equal_split_vectors(mcg, fmt, problem, kw):
    """{r, Ap} stored as 16-B pairs vs separate r / Ap arrays: same arithmetic, same bits."""
    spec = mcg.make_problem(problem, **kw)
    a = mcg.CGSolver(spec, format=fmt, recurrence=1, interleave=1, check_every=8)
    b = mcg.CGSolver(spec, format=fmt, recurrence=1, interleave=0, check_every=8)
    assert a.info["interleave"] and not b.info["interleave"]
    ra, rb = a.solve(), b.solve()
    assert ra["iterations"] == rb["iterations"] and ra["rnorm"] == rb["rnorm"]
    np.testing.assert_array_equal(ra["x_local"], rb["x_local"])


@pytest.mark.parametrize("recurrence", [0, 1])
@pytest.mark.parametrize("problem,kw,plain,expect", [("poisson2d", dict(n=96), "sell16", "sell64-c8"),
                                                    ("poisson3d", dict(n=20), "sell", "sell64-c8"),
                                                    ("randspd", dict(rows=20000, band=40, density=0.25), "sell16",
                                                     "sell64-d16")])
def test_dictionary_codes_bitwise_equal_plain_sell(mcg, recurrence, problem, kw, plain, expect):
    """SELL-64/c8 stores the same entries in the same slot order as SELL-64(/d16): same bits out.
    Matrices with too many distinct (value, offset) pairs fall back to d16."""
    spec = mcg.make_problem(problem, **kw)
    a = mcg.CGSolver(spec, format="sellc8", recurrence=recurrence, check_every=8)
    b = mcg.CGSolver(spec, format=plain, recurrence=recurrence, check_every=8)
    assert a.info["format"] == expect
    ra, rb = a.solve(), b.solve()
    assert ra["iterations"] == rb["iterations"] and ra["rnorm"] == rb["rnorm"]
    np.testing.assert_array_equal(ra["x_local"], rb["x_local"])
    assert a.true_residual_norm() == b.true_residual_norm()


@pytest.mark.parametrize("fmt", ["sell", "sell16"])
@pytest.mark.parametrize("interleave", [0, 1])
def test_window_pass_bitwise_equal_plain(mcg, fmt, interleave):
    """LDS-window pass (p_k staged once per 1024-row chunk) vs per-gather recomputation: the same
    row sums; dot partials are blocked differently, so agreement is to rounding."""
    spec = mcg.make_problem("randspd", rows=30000, band=60, density=0.6)
    a = mcg.CGSolver(spec, format=fmt, recurrence=1, interleave=interleave, window=-1, check_every=8)
    b = mcg.CGSolver(spec, format=fmt, recurrence=1, interleave=interleave, window=0, check_every=8)
    assert a.info["window"] > 0 and b.info["window"] == 0  # mean row length ~73 -> auto on
    ra, rb = a.solve(), b.solve()
    assert ra["converged"] and ra["iterations"] == rb["iterations"]
    assert abs(ra["rnorm"] - rb["rnorm"]) <= 1e-6 * rb["rnorm"]
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-12, atol=1e-15)


def test_window_pass_off_for_stencils(mcg):
    s = mcg.CGSolver(mcg.make_problem("poisson2d", n=256), format="sell16", recurrence=1)
    assert s.info["window"] == 0  # 5 nonzeros per row: per-gather recomputation is cheaper


@pytest.mark.parametrize("fmt", ["sell16", "sellc8"])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=96)), ("poisson3d", dict(n=20))])
def test_pipelined_pass_bitwise_equal_generic(mcg, fmt, problem, kw):
    """Software-pipelined stencil pass vs the generic engine: same arithmetic, same bits."""
    spec = mcg.make_problem(problem, **kw)
    a = mcg.CGSolver(spec, format=fmt, recurrence=1, pipeline=1, check_every=8)
    b = mcg.CGSolver(spec, format=fmt, recurrence=1, pipeline=0, check_every=8)
    assert a.info["pipeline"] and not b.info["pipeline"]
    ra, rb = a.solve(), b.solve()
    assert ra["iterations"] == rb["iterations"] and ra["rnorm"] == rb["rnorm"]
    np.testing.assert_array_equal(ra["x_local"], rb["x_local"])


def test_interleave_requires_single_reduction_sell(mcg):
    with pytest.raises(Exception, match="interleaved"):
        mcg.CGSolver(mcg.make_problem("poisson2d", n=32), format="csr", recurrence=1, interleave=1)


def test_single_reduction_demo_and_maxit(mcg):
    out = mcg.CGSolver(mcg.make_problem("demo"), recurrence=1).solve()
    assert "".join("%f\n" % v for v in out["x_local"]) == "0.500000\n0.750000\n1.000000\n"
    assert out["iterations"] == 3 and out["converged"]
    spec = mcg.make_problem("poisson2d", n=200)
    cpu = mcg.native().cpu_cg(spec.native(), mcg.native().CgOptions(maxit=50, tol=1e-7))
    out = mcg.CGSolver(spec, maxit=50, recurrence=1, format="sell").solve()
    assert out["iterations"] == 50 and not out["converged"]
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-8, atol=1e-12)
    assert abs(out["rnorm"] - cpu["rnorm"]) <= 1e-6 * cpu["rnorm"]


def test_fixed_iterations_counter(mcg):
    spec = mcg.make_problem("poisson2d", n=512)
    s = mcg.CGSolver(spec, tol=-1.0, maxit=1 << 30)
    s.reset()
    s.run(7)
    s.run(10)
    s.synchronize()
    r = s.result()
    assert r["iterations"] == 17 and not r["converged"] and np.isfinite(r["rnorm"])


def test_maxit_exhaustion_matches_cpu(mcg):
    spec = mcg.make_problem("poisson2d", n=200)
    cpu = mcg.native().cpu_cg(spec.native(), mcg.native().CgOptions(maxit=50, tol=1e-7))
    out = mcg.CGSolver(spec, maxit=50, format="csr", recurrence=0).solve()
    assert out["iterations"] == 50 and not out["converged"]
    np.testing.assert_allclose(out["x_local"], cpu["x"], rtol=1e-9, atol=1e-12)
    assert abs(out["rnorm"] - cpu["rnorm"]) <= 1e-8 * cpu["rnorm"]


def test_library_default_is_the_cli_fast_path(mcg):
    """CGSolver / solve() pick what the CLIs pick: the lean three-term line carry
    for a generated 2-D stencil, the reference's CSR two-reduction order for the demo."""
    s = mcg.CGSolver(mcg.make_problem("poisson2d", n=1024))
    i = s.info
    assert i["carry"] and i["ap_recompute"] and i["dia4"] and i["p3"] and i["lean_only"], i
    out = mcg.solve("poisson2d", n=1024, tol=1e-6, maxit=20000)  # 1024^2 needs more than the reference's 2000
    assert out["converged"] and out["rnorm"] <= 1e-6
    d = mcg.CGSolver(mcg.make_problem("demo"))
    assert d.info["recurrence"] == "two-reduction"


def test_force_comm_single_rank(mcg):
    """The RCCL code path with one rank (all-reduce degenerates, no halo)."""
    spec = mcg.make_problem("poisson2d", n=64)
    out = mcg.CGSolver(spec, force_comm=True).solve()
    cpu = mcg.native().cpu_cg(spec.native(), mcg.native().CgOptions())
    assert out["converged"] and abs(out["iterations"] - cpu["iterations"]) <= 2


def test_phase_profile_diagnostic(mcg):
    """Per-phase hipEvent timing of the single-reduction iteration (bench.py check.phase_us)."""
    spec = mcg.make_problem("poisson2d", n=512)
    s = mcg.CGSolver(spec, tol=-1.0, maxit=1 << 30, format="sellc8", recurrence=1, force_comm=True)
    s.reset()
    s.run(4)
    ph = s._s.phase_profile(6)
    assert set(ph) == {"interior_or_all", "halo_side_stream", "boundary_wait", "boundary", "reduce", "allreduce",
                       "iteration"}
    assert ph["iteration"] > 0 and ph["interior_or_all"] > 0 and ph["allreduce"] > 0
    assert ph["iteration"] >= ph["interior_or_all"]
    s.synchronize()
    assert s.result()["iterations"] == 10


@pytest.mark.parametrize("recurrence,fmt", [(0, "csr"), (1, "sellc8")])
def test_relative_tolerance_matches_cpu(mcg, recurrence, fmt):
    spec = mcg.make_problem("poisson2d", n=96)
    C = mcg.native()
    o = C.CgOptions(maxit=2000, tol=1e-30)
    o.rtol = 1e-8
    cpu = C.cpu_cg(spec.native(), o)
    out = mcg.CGSolver(spec, format=fmt, recurrence=recurrence, tol=1e-30, rtol=1e-8, check_every=8).solve()
    assert out["converged"] and abs(out["iterations"] - cpu["iterations"]) <= 2


@pytest.mark.parametrize("fmt", ["sell16", "sellc8"])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=128)), ("poisson2d", dict(n=256)),
                                        ("poisson3d", dict(n=16))])
def test_line_carry_pass_matches_generic(mcg, fmt, problem, kw):
    """Line-carry pass (a wave walks down one slice column; the +-one-line neighbours' p_k stay in
    registers) vs the generic pass: the same per-row arithmetic, dot-product partials blocked
    differently -> fixed-iteration residuals agree to rounding, solutions to the solver tolerance."""
    spec = mcg.make_problem(problem, rhs="random", **kw)
    a = mcg.CGSolver(spec, format=fmt, recurrence=1, carry=1, check_every=8)
    b = mcg.CGSolver(spec, format=fmt, recurrence=1, carry=0, check_every=8)
    assert a.info["carry"] and not b.info["carry"]
    ra, rb = a.solve(), b.solve()
    assert ra["converged"] and rb["converged"] and abs(ra["iterations"] - rb["iterations"]) <= 1
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-6, atol=1e-6 * np.abs(rb["x_local"]).max())
    assert a.true_residual_norm() < 1e-6
    outs = []
    for s in (a, b):
        s.reset()
        s.run(24)
        s.finalize()
        outs.append(s.result())
    assert outs[0]["iterations"] == outs[1]["iterations"] == 24
    assert abs(outs[0]["rnorm"] - outs[1]["rnorm"]) <= 1e-9 * outs[1]["rnorm"]


@pytest.mark.parametrize("n", [64, 128])
def test_plane_carry_block_exchange(mcg, n):
    """3-D store-form plane carry with the +-N rows of a block's inner waves exchanged through LDS vs
    the generic pass: the same p_k values in the same fma order, dot-product partials blocked
    differently.  (The variant where every wave gathers its +-N rows lost and was removed in r3.)"""
    spec = mcg.make_problem("poisson3d", n=n, rhs="random")
    solvers = [mcg.CGSolver(spec, format="sellc8", recurrence=1, carry=c, ap_recompute=0, check_every=8)
               for c in (1, 0)]
    assert [s.info["carry_xchg"] for s in solvers] == [True, False]
    assert [s.info["carry"] for s in solvers] == [True, False]
    res = [s.solve() for s in solvers]
    assert all(r["converged"] for r in res)
    assert abs(res[0]["iterations"] - res[1]["iterations"]) <= 1
    np.testing.assert_allclose(res[0]["x_local"], res[1]["x_local"], rtol=1e-6,
                               atol=1e-6 * np.abs(res[1]["x_local"]).max())
    assert solvers[0].true_residual_norm() < 1e-6
    outs = []
    for s in solvers:
        s.reset()
        s.run(24)
        s.finalize()
        outs.append(s.result())
    assert all(o["iterations"] == 24 for o in outs)
    assert abs(outs[0]["rnorm"] - outs[1]["rnorm"]) <= 1e-9 * outs[1]["rnorm"]
    # run to run: bitwise
    again = mcg.CGSolver(spec, format="sellc8", recurrence=1, carry=1, ap_recompute=0, check_every=8).solve()
    np.testing.assert_array_equal(again["x_local"], res[0]["x_local"])


def test_line_carry_pass_reproducible_and_auto(mcg):
    spec = mcg.make_problem("poisson2d", n=256, rhs="random")
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, carry=-1).solve()
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, carry=-1).solve()
    np.testing.assert_array_equal(a["x_local"], b["x_local"])
    # not applicable (line length not a multiple of 64): auto falls back, on=1 refuses
    odd = mcg.make_problem("poisson2d", n=100)
    assert not mcg.CGSolver(odd, format="sellc8", recurrence=1, carry=-1).info["carry"]
    with pytest.raises(Exception, match="line-carry"):
        mcg.CGSolver(odd, format="sellc8", recurrence=1, carry=1)


@pytest.mark.parametrize("codes", ["dia4", "c8"])
@pytest.mark.parametrize("n", [128, 256])
def test_ap_recompute_bitwise_equal_to_stored_pairs(mcg, codes, n):
    """The line-carry pass that recomputes Ap_{k-1} = A p_{k-1} (same entries, same fma order, same
    p values) instead of storing {r, Ap} pairs: every r, p, x and dot product is the same bits, to
    convergence and at fixed odd / even iteration counts (final pass, paired x updates).  With the
    SELL-64/dia4 storage (slot = canonical offset, absent entries exact zeros) the row sums add the
    same products in the same order, so it is bitwise equal too."""
    spec = mcg.make_problem("poisson2d", n=n, rhs="random")
    dia = 1 if codes == "dia4" else 0
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, carry=1, ap_recompute=1, carry_dia=dia, p3=0, check_every=8)
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, carry=1, ap_recompute=0, check_every=8)
    assert a.info["ap_recompute"] and not a.info["interleave"]
    assert a.info["dia4"] == (codes == "dia4")
    assert not b.info["ap_recompute"] and b.info["interleave"]
    ra, rb = a.solve(), b.solve()
    assert ra["converged"] and ra["iterations"] == rb["iterations"] and ra["rnorm"] == rb["rnorm"]
    np.testing.assert_array_equal(ra["x_local"], rb["x_local"])
    for its in (23, 24):
        outs = []
        for s in (a, b):
            s.reset()
            s.run(its)
            s.finalize()
            outs.append((s.result(), s._s.x_local()))
        assert outs[0][0]["iterations"] == its and outs[0][0]["rnorm"] == outs[1][0]["rnorm"]
        np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert a.true_residual_norm() == b.true_residual_norm()


@pytest.mark.parametrize("problem,n", [("poisson2d", 128), ("poisson2d", 256), ("poisson2d", 512),
                                       ("poisson3d", 64), ("poisson3d", 128)])
def test_three_term_carry_tracks_two_term(mcg, problem, n):
    """Three-term form of the dia4 line carry (r_{k-1} = p_{k-1} - beta p_{k-2} from the two stored p's,
    r kept only at slice edges and run outer lines): the same CG iterates up to rounding -- same
    iteration count (+-1), x and ||r|| to ~1e-9 -- against the two-term form, at convergence and at
    fixed odd / even counts (final pass, paired x updates); the recurrence residual tracks ||b - A x||."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, p3=1, check_every=8)
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, p3=0, check_every=8)
    assert a.info["p3"] and a.info["dia4"] and a.info["ap_recompute"] and not b.info["p3"]
    assert a.info["bytes_per_iter_model"] < b.info["bytes_per_iter_model"]
    ra, rb = a.solve(), b.solve()
    assert ra["converged"] and abs(ra["iterations"] - rb["iterations"]) <= 1
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-7, atol=1e-9 * np.abs(rb["x_local"]).max())
    for its in (23, 24, 101):
        outs = []
        for s in (a, b):
            s.reset()
            s.run(its)
            s.finalize()
            outs.append((s.result(), s._s.x_local()))
        assert outs[0][0]["iterations"] == its
        assert abs(outs[0][0]["rnorm"] - outs[1][0]["rnorm"]) <= 1e-9 * outs[1][0]["rnorm"]
        np.testing.assert_allclose(outs[0][1], outs[1][1], rtol=1e-9, atol=1e-12 * np.abs(outs[1][1]).max())
        tr = a.true_residual_norm()
        assert abs(tr - outs[0][0]["rnorm"]) <= 1e-9 * tr


def test_three_term_carry_refusal(mcg):
    """p3 = 1 where the 2-D dia4 carry does not run: a clear error; auto is on with dia4."""
    assert mcg.CGSolver(mcg.make_problem("poisson2d", n=256), format="sellc8", recurrence=1).info["p3"]
    with pytest.raises(Exception, match="p3"):
        mcg.CGSolver(mcg.make_problem("poisson2d", n=256), format="sellc8", recurrence=1, carry_dia=0, p3=1)


@pytest.mark.parametrize("n", [64, 128])
def test_ap_recompute_3d_matches_store_form(mcg, n):
    """3-D plane carry that recomputes Ap (SELL-64/dia4, +-N rows through LDS between the block's
    kw waves, the outer lines' Ap stored): the same recurrence as the store-form plane carry.  Its runs
    of planes per job column are chosen to fill whole rounds of blocks (carry3_runs), so the
    dot-product partials group differently from the store form's: the same iterations, rounding only
    (kw = 4, pruned in r5, agreed bit for bit while both used one run per column)."""
    spec = mcg.make_problem("poisson3d", n=n, rhs="random")
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, ap_recompute=1, p3=0, check_every=8)
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, ap_recompute=0, check_every=8)
    assert a.info["ap_recompute"] and a.info["dia4"] and a.info["ar3_kw"] == 16
    assert not b.info["ap_recompute"] and b.info["carry"]
    ra, rb = a.solve(), b.solve()
    assert ra["converged"] and abs(ra["iterations"] - rb["iterations"]) <= 1
    if ra["iterations"] == rb["iterations"]:
        assert abs(ra["rnorm"] - rb["rnorm"]) <= 1e-10 * rb["rnorm"]
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-9, atol=1e-12)
    for its in (23, 24):
        outs = []
        for s in (a, b):
            s.reset()
            s.run(its)
            s.finalize()
            outs.append((s.result(), s._s.x_local()))
        assert outs[0][0]["iterations"] == its
        assert abs(outs[0][0]["rnorm"] - outs[1][0]["rnorm"]) <= 1e-11 * outs[1][0]["rnorm"]
        np.testing.assert_allclose(outs[0][1], outs[1][1], rtol=1e-10, atol=1e-13)
    tr = a.true_residual_norm()
    assert abs(tr - outs[0][0]["rnorm"]) <= 1e-8 * tr


def test_ap_recompute_auto_and_refusal(mcg):
    """auto: on for the specialised 2-D carry; off where the carry is off (3-D generic) or the
    rows are not whole 64-row lines; required (=1) where it cannot apply: a clear error."""
    s2 = mcg.CGSolver(mcg.make_problem("poisson2d", n=256), format="sellc8", recurrence=1)
    assert s2.info["ap_recompute"] and s2.info["carry"]
    s3 = mcg.CGSolver(mcg.make_problem("poisson3d", n=32), format="sellc8", recurrence=1)
    assert not s3.info["ap_recompute"]
    with pytest.raises(Exception, match="ap_recompute"):
        mcg.CGSolver(mcg.make_problem("poisson2d", n=100), format="sellc8", recurrence=1, ap_recompute=1)
    assert s2.info["dia4"]  # auto: the 5-pt operator's entries sit at the canonical offsets
    with pytest.raises(Exception, match="carry_dia"):
        mcg.CGSolver(mcg.make_problem("poisson3d", n=32), format="sellc8", recurrence=1, carry_dia=1)


@pytest.mark.parametrize("problem,n", [("poisson2d", 256), ("poisson3d", 40)])
def test_placement_probe_keeps_numerics(mcg, problem, n):
    """The setup-time placement probe (several vector allocations x start offsets, fastest kept) only
    moves where the vectors live: the solve is bitwise equal to one without the probe, and the probe
    leaves no state behind (partials and CgState are cleared)."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, placement_tries=3, placement_leads=4)
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, placement_tries=1)
    assert a.info["placement_sets"] >= 2 and b.info["placement_sets"] == 1
    assert 0 <= a.info["placement_lead_trial"] < 4
    assert a.info["placement_gain"] >= 1.0
    ra, rb = a.solve(), b.solve()
    assert ra["converged"] and rb["converged"] and ra["iterations"] == rb["iterations"]
    assert np.array_equal(ra["x_local"], rb["x_local"])
    assert ra["rnorm"] == rb["rnorm"]


def test_cli_json_report_per_rank_memory(mcg):
    """--report json lists the device bytes each rank's solver holds."""
    import json
    p = subprocess.run([mcg.cli_path(), "--problem", "poisson2d", "--n", "128", "--report", "json"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.strip().splitlines()
    assert lines[-1] == "Success"
    rep = json.loads(lines[-2])
    assert rep["converged"] and rep["ranks"] == 1
    assert rep["device_bytes_per_rank"] == [rep["device_bytes_rank0"]] and rep["device_bytes_rank0"] > 0


@pytest.mark.parametrize("fmt,rec", [("sellc8", 1), ("csr", 0)])
def test_long_graph_bitwise_equal_pairs(mcg, fmt, rec):
    """graph_iters=8 replays 8 iterations per hipGraph launch (the tail as pairs / eagerly); the
    passes depend on k only through its parity, so results are bitwise those of pair graphs."""
    spec = mcg.make_problem("poisson2d", n=96, rhs="random")
    a = mcg.CGSolver(spec, format=fmt, recurrence=rec, graph_iters=8, check_every=32)
    b = mcg.CGSolver(spec, format=fmt, recurrence=rec, graph_iters=2, check_every=32)
    ra, rb = a.solve(), b.solve()
    assert ra["converged"] and ra["iterations"] == rb["iterations"]
    assert np.array_equal(ra["x_local"], rb["x_local"]) and ra["rnorm"] == rb["rnorm"]
    for s in (a, b):
        s.reset()
        s.run(2 + 8 * 3 + 6)  # eager head, long graphs, pair tail
        s.finalize()
    assert a.result()["iterations"] == b.result()["iterations"] == 32
    assert a.result()["rnorm"] == b.result()["rnorm"]
    assert np.array_equal(a.x_local(), b.x_local())


@pytest.mark.parametrize("n", [1024, 2048])
def test_dia_uniform_lean_runs_bitwise(mcg, n):
    """Lean runs of the three-term 2-D dia4 carry (runs whose slices all carry one uniform value
    pattern: values in scalar registers, no codes streamed) compute exactly what the generic step
    computes: x and ||r|| bit for bit against dia_uniform = 0, at odd and even iteration counts
    (paired x update) and at convergence.  Both on one grid of 4 blocks per CU (the auto lean grids
    differ from the generic pass's, and the block partials' order with them): runs of 4 / 16 lines,
    so most runs are lean (l0 >= 2, l1 <= lines - 4)."""
    spec = mcg.make_problem("poisson2d", n=n, rhs="random")
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, check_every=8, blocks_per_cu=4)
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, check_every=8, dia_uniform=0, blocks_per_cu=4)
    assert a.info["p3"] and a.info["dia4"] and b.info["p3"]
    assert a.info["dia_uniform"] > 0.9 and b.info["dia_uniform"] == 0.0
    assert a.info["bytes_per_iter_model"] < b.info["bytes_per_iter_model"]
    for its in (37, 38):
        outs = []
        for s in (a, b):
            s.reset()
            s.run(its)
            s.finalize()
            outs.append((s.result(), s._s.x_local()))
        assert outs[0][0]["rnorm"] == outs[1][0]["rnorm"]
        assert np.array_equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("n", [128, 256])
def test_dia_uniform_lean_runs_bitwise_3d(mcg, n):
    """Lean runs of the 3-D three-term plane carry (per wave: the seven values in scalar registers,
    no codes streamed; the block takes them when every wave's run qualifies): x and ||r|| bit for
    bit against dia_uniform = 0.  Runs of a few planes at n = 128, 64 at n = 256, including the
    grid's first / last planes and the x / y boundary slices."""
    spec = mcg.make_problem("poisson3d", n=n, rhs="random")
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, check_every=8)
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, check_every=8, dia_uniform=0)
    assert a.info["p3"] and a.info["ar3_kw"] == 16 and a.info["dia_uniform"] > 0.99
    for its in (21, 22):
        outs = []
        for s in (a, b):
            s.reset()
            s.run(its)
            s.finalize()
            outs.append((s.result(), s._s.x_local()))
        assert outs[0][0]["rnorm"] == outs[1][0]["rnorm"]
        assert np.array_equal(outs[0][1], outs[1][1])


def test_lean_mix_auto_on_small_grids(mcg):
    """The setup's 2-D lean geometry (r5: every size below 2^29 rows): packed slice edges, the even
    passes on 5 blocks per CU (6 where their runs keep >= 64 lines), the odd passes on their own
    4-per-CU grid at depth 4; the solve tracks the explicitly configured default-kernel solve on the
    same two grids bit for bit.  8192^2 takes 6 per CU for the even passes."""
    spec = mcg.make_problem("poisson2d", n=4096, rhs="random")
    a = mcg.CGSolver(spec, format="sellc8", recurrence=1, check_every=8)
    assert a.info["lean_only"] and a.info["lean_mix"] and a.info["grid_odd"] == a.info["grid_a"] * 4 // 5
    # the same two grids with the default lean kernels (test hook): packed edges are bit for bit those
    b = mcg.CGSolver(spec, format="sellc8", recurrence=1, check_every=8, lean_packed=0)
    assert not b.info["lean_mix"] and b.info["grid_odd"] == a.info["grid_odd"] and b.info["grid_a"] == a.info["grid_a"]
    for its in (15, 38):
        for s in (a, b):
            s.reset()
            s.run(its)
            s.finalize()
        assert a.result()["rnorm"] == b.result()["rnorm"]
        assert np.array_equal(a._s.x_local(), b._s.x_local())
    b.reset()
    assert b._s.phase_profile(8)["iteration"] > 0
    big = mcg.CGSolver(mcg.make_problem("poisson2d", n=8192), format="sellc8", recurrence=1)
    assert big.info["lean_only"] and big.info["lean_mix"] and big.info["grid_odd"] * 6 == big.info["grid_a"] * 4
    assert a.info["grid_odd"] * 5 == a.info["grid_a"] * 4


@pytest.mark.parametrize("n,coef", [(1024, 0), (4096, 0), (1024, 1)])
@pytest.mark.parametrize("graph", [True, False])
def test_p3buf_bitwise_equal_to_two_buffer_lean(mcg, n, coef, graph):
    """Three p buffers (PassForm::p3buf, cg_carry_ar.hip T3): p_k goes to a buffer the pass does not
    read, r is recovered from p_{k-1} / p_{k-2} on every line and the neighbouring slices' edge rows
    are recomputed instead of read from compact edge arrays -- the same sums in the same order, so bit
    for bit the two-buffer lean pass.  41 iterations (an odd count: the final pass's x catch-up), in
    graphs (captures keyed by k mod 3) and eagerly; 4096^2 takes the packed-edge kernels; coef = 1:
    the diav loop (r recovered, the edge rows' Ap still in compact arrays)."""
    spec = mcg.make_problem("poisson2d", n=n, rhs="random", coef=coef)
    outs = {}
    for pb in (1, 0):
        s = mcg.CGSolver(spec, format="sellc8", recurrence=1, tol=-1.0, maxit=41, p3buf=pb, use_graph=graph)
        assert s.info["p3buf"] == (pb == 1) and s.info["lean_only"], s.info
        outs[pb] = (s.solve(), s.true_residual_norm())
    (a, ta), (b, tb) = outs[1], outs[0]
    assert a["rnorm"] == b["rnorm"] and a["iterations"] == b["iterations"] == 41
    np.testing.assert_array_equal(a["x_local"], b["x_local"])
    assert ta == tb


@pytest.mark.parametrize("n,coef", [(128, 0), (256, 0), (128, 1)])
@pytest.mark.parametrize("graph", [True, False])
def test_p3buf_3d_bitwise_equal_to_two_buffer_lean(mcg, n, coef, graph):
    """3-D three p buffers (cg_carry_ar3.hip T3, dia4 and the variable-coefficient diav kernels): r
    recovered from p_{k-1} / p_{k-2} on every plane, the blocks' outer lines and the slices' edge rows,
    none stored -- the same operands in the same fma order as the stored r, so bit for bit the
    two-buffer lean plane carry; 41 iterations."""
    spec = mcg.make_problem("poisson3d", n=n, rhs="random", coef=coef)
    outs = {}
    for pb in (1, 0):
        s = mcg.CGSolver(spec, format="sellc8", recurrence=1, tol=-1.0, maxit=41, p3buf=pb, use_graph=graph)
        assert s.info["p3buf"] == (pb == 1) and s.info["lean_only"], s.info
        outs[pb] = (s.solve(), s.true_residual_norm())
    (a, ta), (b, tb) = outs[1], outs[0]
    assert a["rnorm"] == b["rnorm"] and a["iterations"] == b["iterations"] == 41
    np.testing.assert_array_equal(a["x_local"], b["x_local"])
    assert ta == tb


def test_p3buf_3d_default_converges_like_the_two_buffer_form(mcg):
    """The default 3-D path takes the three buffers and converges to the same x, in the same
    iteration count, as the two-buffer form (latched after an even or an odd pass)."""
    for n in (128, 192):  # the 3-D carry: N a multiple of 64
        spec = mcg.make_problem("poisson3d", n=n, rhs="random")
        s = mcg.CGSolver(spec, format="sellc8", recurrence=-1, rtol=1e-8, maxit=20000)
        assert s.info["p3buf"], s.info
        out = s.solve()
        ref = mcg.CGSolver(spec, format="sellc8", recurrence=-1, rtol=1e-8, maxit=20000, p3buf=0).solve()
        assert out["converged"] and out["iterations"] == ref["iterations"]
        np.testing.assert_array_equal(out["x_local"], ref["x_local"])


def test_p3buf_default_converges_like_the_cpu_oracle(mcg):
    """The default 2-D path takes the three buffers, converges in the oracle's iteration count and
    latches the same x as the two-buffer form (convergence after an even and an odd pass)."""
    C = mcg.native()
    for n in (1024, 768):
        spec = mcg.make_problem("poisson2d", n=n, rhs="random")
        s = mcg.CGSolver(spec, format="sellc8", recurrence=-1, rtol=1e-8, maxit=20000)
        assert s.info["p3buf"], s.info
        out = s.solve()
        ref = mcg.CGSolver(spec, format="sellc8", recurrence=-1, rtol=1e-8, maxit=20000, p3buf=0).solve()
        assert out["converged"] and out["iterations"] == ref["iterations"], (out["iterations"], ref["iterations"])
        np.testing.assert_array_equal(out["x_local"], ref["x_local"])
        co = C.CgOptions(maxit=20000)
        co.rtol = 1e-8
        cpu = C.cpu_cg(spec.native(), co)
        assert abs(out["iterations"] - cpu["iterations"]) <= max(2, cpu["iterations"] // 200)
