"""CU-masked compute stream (CgOptions.reserve_cus, profiles/r3_cumask_probe.md): the solver on the
CUs left by the mask solves the same system, and the mask really leaves one CU per shader engine free
(a masked hog grid never lands on them; a fat side-stream wave does)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("problem,n", [("poisson2d", 1024), ("poisson3d", 64)])
def test_reserve_cus_same_solve(mcg, problem, n):
    """reserve_cus = 32 sizes the grids for 224 CUs: the block partials sum in another order, so the
    iterates agree to rounding (not bitwise) over 300 fixed iterations."""
    spec = mcg.make_problem(problem, n=n)
    kw = dict(format="sellc8", recurrence=1, check_every=8, maxit=300, tol=-1.0)
    a = mcg.CGSolver(spec, **kw).solve()
    b = mcg.CGSolver(spec, reserve_cus=32, **kw).solve()
    assert a["iterations"] == b["iterations"] == 300
    scale = np.abs(a["x_local"]).max()
    np.testing.assert_allclose(b["x_local"], a["x_local"], rtol=0, atol=1e-10 * scale)


def test_reserve_cus_bounds(mcg):
    spec = mcg.make_problem("poisson2d", n=128)
    with pytest.raises(Exception, match="reserve_cus"):
        mcg.CGSolver(spec, format="sellc8", recurrence=1, reserve_cus=200).solve()


def test_masked_hog_leaves_one_cu_per_engine(mcg):
    """The mask's top 32 bits are one CU of every shader engine: a grid of 4 blocks per enabled CU on
    the masked stream uses exactly the other 224 CUs, spread 28 per XCD."""
    import torch

    K = mcg.native().kernels
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    if ncu != 256:
        pytest.skip("mask layout measured on the 256-CU MI355X")
    words = [0xFFFFFFFF] * 7 + [0]
    st = K.cu_mask_stream(words)
    try:
        blocks = 4 * 224
        where = torch.full((blocks,), -1, dtype=torch.int32, device="cuda")
        out = torch.zeros(blocks, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        K.hog(out.data_ptr(), 200.0, blocks, st, where.data_ptr())
        torch.cuda.synchronize()
        used = set(where.tolist())
        assert -1 not in used
        assert len(used) == 224
        per_xcd = {}
        for smid in used:  # __smid = xcc << 6 | se << 4 | cu
            per_xcd[smid >> 6] = per_xcd.get(smid >> 6, 0) + 1
        assert sorted(per_xcd.values()) == [28] * 8
    finally:
        torch.cuda.synchronize()
        K.stream_destroy(st)


def test_cli_reserve_cus(mcg):
    """The native CLI takes --reserve-cus (shared flag table) and solves on the masked stream."""
    import json
    import subprocess

    p = subprocess.run([mcg.cli_path(), "--problem", "poisson2d", "--n", "128", "--format", "sellc8",
                        "--reserve-cus", "32", "--report", "json"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    rep = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rep["converged"]
