"""Stencil ranks past 2^29 rows: the lean line / plane carries re-base their
64-bit pointers per run (2-D) or along the run (3-D) and keep 32-bit byte offsets, so a rank of
more than 2^29 rows (4 GiB per vector) still runs the lean-only kernels (the reference's limit is
int32 indices, CUDACG.cu:213-216; the north star's is 288 GB per GPU).

Each case is checked bit for bit against the generic kernels (dia_uniform = 0: no lean loop, plain
64-bit indexing) over a few fixed iterations."""
import gc

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(mcg, spec, iters, **kw):
    s = mcg.CGSolver(spec, format="sellc8", recurrence=1, tol=-1.0, maxit=iters, check_every=iters, **kw)
    info = dict(s.info)
    out = s.solve()
    x = out["x_local"][:: 4099].copy()  # a sample: the vectors are 4+ GiB
    del s, out
    gc.collect()
    return info, x


@pytest.mark.parametrize("problem,n", [("poisson2d", 23232), ("poisson3d", 832)])
def test_lean_carry_past_2_29_rows_matches_generic(mcg, problem, n):
    spec = mcg.make_problem(problem, n=n, rhs="random")
    assert spec.n_rows > (1 << 29)
    iters = 6
    # the 2-D lean grid on the generic kernels' grid (8 blocks per CU), so the block partials -- and
    # with them the dot products' rounding -- are the same and the comparison is bit for bit
    kw = dict(blocks_per_cu=8) if problem == "poisson2d" else {}
    info_l, x_l = _run(mcg, spec, iters, **kw)
    assert info_l["lean_only"] and info_l["p3"] and info_l["ap_recompute"], info_l
    assert info_l["ext_len"] >= (1 << 29)
    info_g, x_g = _run(mcg, spec, iters, dia_uniform=0)
    assert not info_g["lean_only"] and info_g["grid_a"] == info_l["grid_a"], (info_g["grid_a"], info_l["grid_a"])
    np.testing.assert_array_equal(x_l, x_g)
