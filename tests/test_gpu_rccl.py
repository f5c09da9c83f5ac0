"""Real RCCL across >= 2 GPUs: every collective of csrc/gpu/comm.cpp (the scalar
all-reduce, the grouped halo send/recv on the second communicator, the all-gather ghost
path, async-error polling) through all three launch routes — the native CLI's thread per
GPU, bench.py's process-per-GPU launcher, and the Python CLI under the same launcher.

Skipped when fewer than 2 GPUs are visible (the 1-GPU development pool); the driver's
8-GPU node runs it.  Reference anchor: the reductions at CUDACG.cu:304,328 become the
all-reduce, the SpMV's neighbour reads (:288) the halo.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ngpus():
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


NG = _ngpus()
needs2 = pytest.mark.skipif(NG < 2, reason="needs >= 2 GPUs (RCCL refuses two ranks on one device)")
WORLDS = [p for p in (2, 4, 8) if p <= max(NG, 2)]

PROBLEMS = {
    "poisson2d": ["--problem", "poisson2d", "--n", "96"],
    "poisson3d": ["--problem", "poisson3d", "--n", "20"],
    "randspd": ["--problem", "randspd", "--rows", "20000", "--band", "40", "--density", "0.25"],
    "randspd_wide": ["--problem", "randspd", "--rows", "20000", "--band", "24", "--density", "0.5", "--spread",
                     "20000"],
}


def _cpu_x(mcg, args):
    p = subprocess.run([mcg.cli_path(), "--device", "cpu", "--print-x", "yes", "--report", "json"] + args,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout
    lines = p.stdout.splitlines()
    return np.array([float(v) for v in lines[:-2]]), json.loads(lines[-2])


def _run(cmd, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


@needs2
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("problem", sorted(PROBLEMS))
@pytest.mark.parametrize("mode", [["--recurrence", "single"], ["--recurrence", "two"],
                                  ["--recurrence", "single", "--no-overlap"], ["--recurrence", "single", "--no-graph"]])
def test_native_cli_threads_match_cpu(mcg, world, problem, mode):
    args = PROBLEMS[problem]
    x_cpu, rep_cpu = _cpu_x(mcg, args)
    p = _run([mcg.cli_path(), "--gpus", str(world), "--print-x", "yes", "--report", "json", "--verify",
              "--watchdog", "120", "--format", "sell"] + mode + args)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = p.stdout.splitlines()
    rep = json.loads(lines[-2])
    x = np.array([float(v) for v in lines[:-2]])
    assert rep["ranks"] == world and rep["converged"]
    assert abs(rep["iterations"] - rep_cpu["iterations"]) <= max(2, rep_cpu["iterations"] // 100)
    assert rep["true_rnorm"] < 1e-6
    np.testing.assert_allclose(x, x_cpu, atol=2e-6 * np.abs(x_cpu).max())  # %f output resolution


@needs2
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("args", [["--problem", "poisson2d", "--n", "128"], ["--problem", "poisson3d", "--n", "64"]])
@pytest.mark.parametrize("mode", [[], ["--no-graph"]])
def test_native_cli_threads_carry_paths_match_cpu(mcg, world, args, mode):
    """The default stencil path at P > 1 over real RCCL: dia4 line / plane carry in the three-term
    form, halo ahead of the pass (r, Ap, p of the ghost lines), graphs with the collectives."""
    x_cpu, rep_cpu = _cpu_x(mcg, args)
    p = _run([mcg.cli_path(), "--gpus", str(world), "--print-x", "yes", "--report", "json", "--verify",
              "--watchdog", "120"] + mode + args)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = p.stdout.splitlines()
    rep = json.loads(lines[-2])
    x = np.array([float(v) for v in lines[:-2]])
    assert rep["ranks"] == world and rep["converged"]
    assert abs(rep["iterations"] - rep_cpu["iterations"]) <= max(2, rep_cpu["iterations"] // 100)
    assert rep["true_rnorm"] < 1e-6
    np.testing.assert_allclose(x, x_cpu, atol=2e-6 * np.abs(x_cpu).max())


@needs2
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("problem", ["poisson2d", "randspd_wide"])
def test_bench_launcher_processes(world, problem):
    """bench.py --gpus P starts P processes; all ranks agree and the true residual matches."""
    extra = (["--grid", "512"] if problem == "poisson2d"
             else ["--problem", "randspd", "--rows", "200000", "--band", "64", "--density", "0.5"])
    p = _run([sys.executable, "bench.py", "--gpus", str(world), "--steps", "40", "--warmup", "5"] + extra)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["check"]["comm_world"] == world
    assert line["check"]["ok"] and line["config"]["launch"] == "spawn"
    assert line["check"]["graph_fallbacks"] == 0


@needs2
@pytest.mark.parametrize("world", WORLDS)
def test_bench_matches_single_gpu_fixed_iterations(world):
    """Same fixed iterations at P = 1 and P: the recurrence residual agrees to rounding."""
    out = []
    for p_ in (1, world):
        p = _run([sys.executable, "bench.py", "--gpus", str(p_), "--grid", "1024", "--steps", "100", "--warmup", "0",
                  "--phases", "0"])
        assert p.returncode == 0, p.stdout + p.stderr
        out.append(json.loads(p.stdout.strip().splitlines()[-1]))
    r1, rp = out[0]["check"]["rnorm"], out[1]["check"]["rnorm"]
    assert abs(r1 - rp) <= 1e-9 * r1


@needs2
@pytest.mark.parametrize("world", WORLDS[:1])
def test_python_cli_processes(mcg, world):
    args = PROBLEMS["poisson2d"]
    x_cpu, rep_cpu = _cpu_x(mcg, args)
    p = _run([sys.executable, "-m", "cuda_mpi_parallel_amd", "--gpus", str(world), "--print-x", "yes",
              "--report", "json", "--verify"] + args)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = p.stdout.splitlines()
    rep = json.loads(lines[-2])
    assert rep["ranks"] == world and rep["true_rnorm"] < 1e-6
    x = np.array([float(v) for v in lines[:-2]])
    np.testing.assert_allclose(x, x_cpu, atol=2e-6 * np.abs(x_cpu).max())


@needs2
def test_nan_injection_latches_every_rank(mcg):
    p = _run([mcg.cli_path(), "--gpus", "2", "--report", "json", "--inject-nan-at", "5", "--watchdog", "60"]
             + PROBLEMS["poisson2d"])
    assert p.returncode == 0, p.stdout + p.stderr
    rep = json.loads(p.stdout.splitlines()[-2])
    assert rep["breakdown"] and not rep["converged"]


def test_single_gpu_pool_skips_cleanly():
    """On one GPU this module only checks that the launchers refuse P > devices, fast."""
    if NG >= 2:
        pytest.skip("multi-GPU node: the real tests above ran")
    p = _run([sys.executable, "bench.py", "--gpus", "2"], timeout=120)
    assert p.returncode == 2 and "--gpus 2" in p.stderr


def _one_rank_comm(mcg):
    C = mcg.native()
    return C.Comm(0, 1, C.unique_id(), C.unique_id())


@pytest.mark.parametrize("graph", [False, True])
def test_rccl_loopback_sendrecv_and_allgather_on_one_gpu(mcg, graph):
    """On one GPU the grouped ncclSend/ncclRecv (to this rank) and the in-place ncclAllGather run
    through the same Comm calls the halo uses, eager and captured into a hipGraph."""
    import torch

    torch.cuda.set_device(0)
    comm = _one_rank_comm(mcg)
    n = 1 << 16
    a = torch.arange(n, dtype=torch.float64, device="cuda") * 0.5
    b = torch.zeros_like(a)
    g = torch.arange(n, dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()

    def step():
        comm.sendrecv_ptr(a.data_ptr(), 0, b.data_ptr(), 0, n, s.cuda_stream)
        comm.allgather_inplace_ptr(g.data_ptr(), n, s.cuda_stream)

    if graph:
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            cg.capture_begin()
            step()
            cg.capture_end()
        b.zero_()
        torch.cuda.synchronize()
        cg.replay()
        cg.replay()
    else:
        with torch.cuda.stream(s):
            step()
    torch.cuda.synchronize()
    comm.check_async()
    assert torch.equal(b, a)
    assert torch.equal(g, torch.arange(n, dtype=torch.float64, device="cuda"))
