"""One kernel per iteration: the fused pass reduces its own block partials (kernels.hpp RedCtl),
hipGraph behaviour around it, and long-run parity of the GPU recurrences with the CPU oracle.

Reference anchors: the two blocking reductions per iteration, CUDACG.cu:304 (p.Ap) and :328
(||r||), become one in-kernel fan-in + one 32-B all-reduce; the stop test :333 and the
recurrence :311-351 must survive 2000 iterations (the reference's maxit, :244).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [
    # (problem, spec kwargs, solver kwargs): the line-carry pass, the generic SELL/c8 pass, the
    # pipelined pass (3-D), plain CSR, the windowed pass (long banded rows)
    ("poisson2d", dict(n=128), dict(format="sellc8")),
    ("poisson2d", dict(n=96), dict(format="sell16", carry=0)),
    ("poisson3d", dict(n=24), dict(format="sellc8")),
    ("poisson2d", dict(n=96), dict(format="csr")),
    ("randspd", dict(rows=20000, band=200, density=0.3), dict(format="sell16", window=1)),
]


def _solver(mcg, problem, kw, skw, **extra):
    spec = mcg.make_problem(problem, **kw)
    return mcg.CGSolver(spec, recurrence=1, check_every=8, **{**skw, **extra})


@pytest.mark.parametrize("problem,kw,skw", CASES)
def test_fused_reduce_matches_separate_reduce(mcg, problem, kw, skw):
    a = _solver(mcg, problem, kw, skw, fused_reduce=-1)
    b = _solver(mcg, problem, kw, skw, fused_reduce=0)
    assert a.info["fused_reduce"] and not b.info["fused_reduce"]
    ra, rb = a.solve(), b.solve()
    # the two reductions sum the same block partials in different fixed orders
    assert abs(ra["iterations"] - rb["iterations"]) <= 1
    assert ra["converged"] and rb["converged"]
    np.testing.assert_allclose(ra["x_local"], rb["x_local"], rtol=1e-8, atol=1e-10 * np.abs(rb["x_local"]).max())
    assert a.true_residual_norm() < 1e-6


@pytest.mark.parametrize("problem,kw,skw", CASES)
def test_fused_reduce_bitwise_repeatable_and_graph_equals_eager(mcg, problem, kw, skw):
    """Fixed-order fan-in: the same bits however the blocks are scheduled, graph or eager."""
    outs = []
    for graph in (True, True, False):
        s = _solver(mcg, problem, kw, skw, use_graph=graph)
        outs.append(s.solve())
    for o in outs[1:]:
        assert o["iterations"] == outs[0]["iterations"] and o["rnorm"] == outs[0]["rnorm"]
        np.testing.assert_array_equal(o["x_local"], outs[0]["x_local"])


def test_fixed_iterations_fused_vs_separate_long_run(mcg):
    """400 fixed iterations (no latch) at 512^2: the two reductions stay within rounding."""
    spec = mcg.make_problem("poisson2d", n=512, rhs="random")
    res = []
    for fr in (-1, 0):
        s = mcg.CGSolver(spec, recurrence=1, tol=-1.0, maxit=400, format="sellc8", fused_reduce=fr)
        out = s.solve()
        assert out["iterations"] == 400
        res.append(out)
    assert abs(res[0]["rnorm"] - res[1]["rnorm"]) <= 1e-10 * res[1]["rnorm"]


def test_graph_launch_failure_falls_back_bitwise(mcg):
    """A graph launch that reports a pre-enqueue error: the solver runs those iterations eagerly,
    exactly once (no double application of x / r / p updates)."""
    spec = mcg.make_problem("poisson2d", n=96)
    eager = mcg.CGSolver(spec, recurrence=1, use_graph=False, check_every=8).solve()
    s = mcg.CGSolver(spec, recurrence=1, use_graph=True, check_every=8, fail_graph_launch_at=8)
    out = s.solve()
    assert s.info["graph_fallbacks"] == 1
    assert out["iterations"] == eager["iterations"] and out["rnorm"] == eager["rnorm"]
    np.testing.assert_array_equal(out["x_local"], eager["x_local"])


@pytest.mark.parametrize("fused", [-1, 0])
def test_rccl_allreduce_captured_in_graph(mcg, fused):
    """force_comm at one rank: the RCCL all-reduce of the 4 sums is captured into the iteration
    graphs (the P > 1 default) and gives the same bits as the communicator-free run."""
    spec = mcg.make_problem("poisson2d", n=128)
    plain = mcg.CGSolver(spec, recurrence=1, use_graph=True, fused_reduce=fused, check_every=8).solve()
    s = mcg.CGSolver(spec, recurrence=1, use_graph=True, fused_reduce=fused, check_every=8, force_comm=True)
    out = s.solve()
    assert s.info["graph_fallbacks"] == 0
    assert out["iterations"] == plain["iterations"] and out["rnorm"] == plain["rnorm"]
    np.testing.assert_array_equal(out["x_local"], plain["x_local"])


@pytest.fixture(scope="module")
def cpu_2000(mcg):
    """CPU oracle at BASELINE config 1's size: 1024^2 5-pt Poisson, 2000 iterations, no stop."""
    C = mcg.native()
    spec = mcg.make_problem("poisson2d", n=1024, rhs="random")
    return spec, C.cpu_cg(spec.native(), C.CgOptions(maxit=2000, tol=-1.0))


@pytest.mark.parametrize("recurrence", [0, 1])
def test_2000_iterations_track_cpu_oracle(mcg, cpu_2000, recurrence):
    """Residual every 250th iteration and the final x against the CPU reference recurrence
    (op-for-op CUDACG.cu:269-352) over the reference's full maxit."""
    spec, cpu = cpu_2000
    hist = np.asarray(cpu["rnorm_history"])
    assert len(hist) == 2000
    fmt = "csr" if recurrence == 0 else "sellc8"
    worst = 0.0
    for m in range(250, 2001, 250):
        s = mcg.CGSolver(spec, recurrence=recurrence, tol=-1.0, maxit=m, format=fmt)
        out = s.solve()
        assert out["iterations"] == m
        rel = abs(out["rnorm"] - hist[m - 1]) / hist[m - 1]
        worst = max(worst, rel)
        assert rel <= 1e-9, (m, out["rnorm"], hist[m - 1])
        if recurrence == 1:
            assert out["beta_clamps"] == 0  # the expanded ||r - a Ap||^2 never went non-positive
    x = s.x_local()
    np.testing.assert_allclose(x, cpu["x"], rtol=1e-9, atol=1e-9 * np.abs(cpu["x"]).max())
    print(f"recurrence {recurrence}: worst residual-history gap {worst:.3e}")
