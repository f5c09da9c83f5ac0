"""Auxiliary subsystems on the GPU: checkpoint/resume, fault injection / breakdown
detection, int64 row pointers, race detection (serialised vs. concurrent launch
order must give bitwise-identical results), roctx tracing."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("recurrence,pipe_rr", [(0, 0), (1, 0), (2, 0), (2, 12)])
def test_checkpoint_resume_matches_uninterrupted(mcg, tmp_path, recurrence, pipe_rr):
    """Resume is bitwise equal to the uninterrupted solve for every recurrence (pipelined CG: the
    w, s, z, q vectors, the local {gamma, delta} and the replacement schedule continue)."""
    spec = mcg.make_problem("poisson2d", n=128)
    kw = dict(recurrence=recurrence, format="sell16", check_every=8)
    if recurrence == 2:
        kw["pipe_rr"] = pipe_rr
    full = mcg.CGSolver(spec, **kw).solve()
    # first leg: stop at maxit=40 with a checkpoint every 16 iterations
    prefix = str(tmp_path / "ckpt")
    a = mcg.CGSolver(spec, maxit=40, checkpoint_every=16, checkpoint_path=prefix, **kw)
    a.solve()
    assert os.path.exists(prefix + ".rank0")
    # second leg: fresh solver (new process state), resume from the last checkpoint
    b = mcg.CGSolver(spec, **kw)
    b.load_checkpoint(prefix)
    out = b.solve(resume=True)
    assert out["converged"] and out["iterations"] == full["iterations"]
    np.testing.assert_array_equal(out["x_local"], full["x_local"])


@pytest.mark.parametrize("problem,n,every", [("poisson2d", 1024, 50), ("poisson3d", 128, 50)])
def test_checkpoint_resume_three_p_buffers(mcg, tmp_path, problem, n, every):
    """Three p buffers (p_j in p_[j mod 3]): a checkpoint taken at an iteration that is not a multiple of
    3 (the buffer rotation mid-cycle) resumes bitwise equal to the uninterrupted solve, 2-D and 3-D."""
    spec = mcg.make_problem(problem, n=n, rhs="random")
    kw = dict(format="sellc8", recurrence=1, check_every=8, maxit=400)
    full = mcg.CGSolver(spec, **kw).solve()
    prefix = str(tmp_path / "ck")
    a = mcg.CGSolver(spec, checkpoint_every=every, checkpoint_path=prefix, **dict(kw, maxit=2 * every + 7))
    assert a.info["p3buf"], a.info
    a.solve()
    b = mcg.CGSolver(spec, **kw)
    b.load_checkpoint(prefix)
    out = b.solve(resume=True)
    assert out["iterations"] == full["iterations"] and out["rnorm"] == full["rnorm"]
    np.testing.assert_array_equal(out["x_local"], full["x_local"])


@pytest.mark.parametrize("p3", [0, 1])
def test_checkpoint_resume_default_stencil_path(mcg, tmp_path, p3):
    """The default stencil path (dia4 line carry, Ap recomputed; p3 = three-term form, whose r lives
    only at edge rows / run outer lines and whose beta_{k-2} is in CgState): resume is bitwise equal
    to the uninterrupted solve; a checkpoint of the other pass form is refused."""
    spec = mcg.make_problem("poisson2d", n=256, rhs="random")
    kw = dict(format="sellc8", recurrence=1, p3=p3, check_every=8)
    full = mcg.CGSolver(spec, **kw).solve()
    prefix = str(tmp_path / "ck")
    a = mcg.CGSolver(spec, maxit=120, checkpoint_every=48, checkpoint_path=prefix, **kw)
    assert a.info["p3"] == bool(p3) and a.info["ap_recompute"]
    a.solve()
    b = mcg.CGSolver(spec, **kw)
    b.load_checkpoint(prefix)
    out = b.solve(resume=True)
    assert out["converged"] and out["iterations"] == full["iterations"] and out["rnorm"] == full["rnorm"]
    np.testing.assert_array_equal(out["x_local"], full["x_local"])
    other = mcg.CGSolver(spec, **dict(kw, p3=1 - p3))
    with pytest.raises(Exception, match="does not match"):
        other.load_checkpoint(prefix)


def test_checkpoint_rejects_other_problem(mcg, tmp_path):
    prefix = str(tmp_path / "c")
    s = mcg.CGSolver(mcg.make_problem("poisson2d", n=64), maxit=5)
    s.solve()
    s.save_checkpoint(prefix)
    t = mcg.CGSolver(mcg.make_problem("poisson2d", n=32))
    with pytest.raises(Exception, match="does not match"):
        t.load_checkpoint(prefix)


def test_checkpoint_rejects_perturbed_user_matrix_or_rhs(mcg, tmp_path):
    """Checkpoint v3 records a fingerprint of the user matrix (rowptr / cols / vals) and of b: a
    resume against a matrix of the same size and pattern with one value changed, or against the
    same matrix with another right-hand side, is refused; the unchanged problem resumes."""
    import scipy.sparse as sp

    n = 400
    T = sp.diags([-1.0, 2.5, -1.0], [-1, 0, 1], shape=(n, n)).tocsr()
    b = np.linspace(0.0, 1.0, n)
    prefix = str(tmp_path / "u")
    kw = dict(format="sell16", recurrence=1, check_every=4)
    a = mcg.CGSolver(mcg.csr_problem(T, b=b), maxit=8, **kw)
    a.solve()
    a.save_checkpoint(prefix)
    mcg.CGSolver(mcg.csr_problem(T, b=b), **kw).load_checkpoint(prefix)  # same problem: accepted
    T2 = T.copy()
    T2.data[7] += 1e-3
    with pytest.raises(Exception, match="does not match"):
        mcg.CGSolver(mcg.csr_problem(T2, b=b), **kw).load_checkpoint(prefix)
    with pytest.raises(Exception, match="does not match"):
        mcg.CGSolver(mcg.csr_problem(T, b=b + 1.0), **kw).load_checkpoint(prefix)


@pytest.mark.parametrize("recurrence,fmt", [(0, "csr"), (1, "csr"), (1, "sell16"), (1, "sellc8"), (2, "sell16")])
def test_fault_injection_latches_breakdown(mcg, recurrence, fmt):
    spec = mcg.make_problem("poisson2d", n=64)
    out = mcg.CGSolver(spec, recurrence=recurrence, format=fmt, inject_nan_at=5, check_every=4).solve()
    assert out["breakdown"] and not out["converged"]
    assert out["iterations"] <= 8


def test_int64_row_pointers(mcg):
    spec = mcg.make_problem("randspd", rows=20000, band=40, density=0.25)
    a = mcg.CGSolver(spec, format="csr").solve()
    b = mcg.CGSolver(spec, format="csr", force_idx64=1).solve()
    assert a["iterations"] == b["iterations"]
    np.testing.assert_array_equal(a["x_local"], b["x_local"])


_RUN = r"""
import json, sys
sys.path.insert(0, %r)
import torch, numpy as np
import cuda_mpi_parallel_amd as m
torch.cuda.set_device(0)
s = m.CGSolver(m.make_problem("poisson2d", n=96), format="sell16", check_every=4, recurrence=%d)
out = s.solve()
print(json.dumps({"it": out["iterations"], "x": out["x_local"].tolist()}))
"""


@pytest.mark.parametrize("recurrence", [0, 1, 2])
def test_serialised_launches_bitwise_identical(mcg, recurrence):
    """Race detection: AMD_SERIALIZE_KERNEL=3 (+ blocking launches) must not change one bit."""
    code = _RUN % (ROOT, recurrence)
    normal = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3", HIP_LAUNCH_BLOCKING="1")
    serial = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert normal.returncode == 0, normal.stderr
    assert serial.returncode == 0, serial.stderr
    a = json.loads(normal.stdout.strip().splitlines()[-1])
    b = json.loads(serial.stdout.strip().splitlines()[-1])
    assert a["it"] == b["it"] and a["x"] == b["x"]


def test_run_to_run_bitwise_reproducible(mcg):
    spec = mcg.make_problem("poisson3d", n=24)
    a = mcg.CGSolver(spec, format="sell16").solve()
    b = mcg.CGSolver(spec, format="sell16").solve()
    np.testing.assert_array_equal(a["x_local"], b["x_local"])


def test_roctx_tracing_enabled_run(mcg):
    code = _RUN % (ROOT, 0)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MCG_TRACE="1"))
    assert p.returncode == 0, p.stderr


def test_watchdog_bounded_wait(mcg):
    """--watchdog: a poll interval that makes no progress within the bound fails loudly; a
    generous bound changes nothing."""
    spec = mcg.make_problem("poisson2d", n=2048)
    ok = mcg.CGSolver(spec, maxit=64, check_every=16, watchdog_seconds=600.0).solve()
    ref = mcg.CGSolver(spec, maxit=64, check_every=16).solve()
    assert ok["iterations"] == ref["iterations"] == 64 and ok["rnorm"] == ref["rnorm"]
    with pytest.raises(Exception, match="watchdog"):
        mcg.CGSolver(spec, maxit=2000, check_every=256, watchdog_seconds=1e-9, use_graph=False).solve()
