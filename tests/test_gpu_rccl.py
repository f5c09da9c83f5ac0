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
@pytest.mark.parametrize("comm", ["dual", "single"])
def test_native_cli_threads_carry_paths_match_cpu(mcg, world, args, mode, comm):
    """The default stencil path at P > 1 over real RCCL: dia4 line / plane carry in the three-term
    form, halo ahead of the pass (r, Ap, p of the ghost lines), graphs with the collectives; with
    two communicators (halo on the side stream) and with one (every collective on the compute
    stream, in one order)."""
    x_cpu, rep_cpu = _cpu_x(mcg, args)
    p = _run([mcg.cli_path(), "--gpus", str(world), "--print-x", "yes", "--report", "json", "--verify",
              "--watchdog", "120", "--comm", comm] + mode + args)
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
@pytest.mark.parametrize("problem", ["poisson2d", "randspd_wide", "randspd_scrambled"])
@pytest.mark.parametrize("comm", ["dual", "single"])
def test_bench_launcher_processes(world, problem, comm):
    """bench.py --gpus P starts P processes; all ranks agree and the true residual matches."""
    extra = (["--grid", "512"] if problem == "poisson2d"
             else ["--problem", "randspd", "--rows", "200000", "--band", "64", "--density", "0.5"]
             + (["--scramble", "1"] if problem == "randspd_scrambled" else []))
    p = _run([sys.executable, "bench.py", "--gpus", str(world), "--steps", "40", "--warmup", "5", "--comm", comm]
             + extra)
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
@pytest.mark.parametrize("world", WORLDS)
def test_bench_default_transport_probed_and_matches_one_gpu(world):
    """the default P > 1 path at a lean size (4096^2: 512 lines a rank at P = 8),
    and which transport it took.  The transport probe must have run on the real fabric, found the
    pulled run bit for bit the exchanged one and the IPC all-reduce's sums RCCL's to rounding, and kept
    the faster of each (its choice is in the JSON); the fixed-iteration residual matches one GPU.  With
    the probe off the verified pull runs (the r5 default), with --halo-transport rccl the exchange: both
    match as well."""
    # 4096^2: 512 lines a rank at P = 8, long enough runs for the lean carry (and so for the pull)
    args = ["--grid", "4096", "--steps", "60", "--warmup", "4", "--phases", "0", "--watchdog", "120"]
    out = {}
    for tag, extra in (("one", ["--gpus", "1"]), ("auto", ["--gpus", str(world)]),
                       ("noprobe", ["--gpus", str(world), "--set", "transport_probe=0"]),
                       ("rccl", ["--gpus", str(world), "--halo-transport", "rccl", "--allreduce", "rccl"])):
        p = _run([sys.executable, "bench.py"] + extra + args)
        assert p.returncode == 0, (tag, p.stdout + p.stderr)
        out[tag] = json.loads(p.stdout.strip().splitlines()[-1])
        assert out[tag]["check"]["ok"] and out[tag]["check"]["graph_fallbacks"] == 0, (tag, out[tag]["check"])
    pr = out["auto"]["check"]["transport_probe"]
    assert pr["pull_bitwise"] and pr["ipc_ar_close"] and not pr.get("ipc_ar_timeout"), pr
    assert out["auto"]["check"]["halo_pull"] == pr["chosen"].startswith("pull")
    assert out["auto"]["config"]["allreduce"].startswith("ipc") == pr["chosen"].endswith("ipc")
    assert out["noprobe"]["check"]["halo_pull"] and "transport_probe" not in out["noprobe"]["check"]
    assert out["noprobe"]["config"]["halo_transport"].startswith("in-kernel")
    assert not out["rccl"]["check"]["halo_pull"]
    r1 = out["one"]["check"]["rnorm"]
    for tag in ("auto", "noprobe", "rccl"):
        assert abs(out[tag]["check"]["rnorm"] - r1) <= 1e-12 * r1, (tag, out[tag]["check"]["rnorm"], r1)


@needs2
@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("problem", [["--problem", "poisson2d", "--n", "4096"], ["--problem", "poisson3d", "--n", "128"]])
def test_native_cli_threads_default_path_reports_transport(mcg, world, problem):
    """bin/mcg-cg --gpus P: each rank thread maps its neighbours' buffers (plain pointers, peer access)
    and every rank's IPC mailbox; the probe's choice is reported and the solve matches one GPU."""
    fixed = ["--fixed-iters", "40", "--report", "json", "--print-x", "no", "--watchdog", "120"]
    one = json.loads(_run([mcg.cli_path()] + problem + fixed).stdout.splitlines()[-2])
    p = _run([mcg.cli_path(), "--gpus", str(world)] + problem + fixed)
    assert p.returncode == 0, p.stdout + p.stderr
    rep = json.loads(p.stdout.splitlines()[-2])
    pr = rep["transport_probe"]
    # (the halo arms run where every rank's pass is the lean carry: not on 16-plane ranks of 128^3 at P = 8)
    assert pr is not None and (pr["pull_us"] == 0 or pr["pull_bitwise"]) and pr["ipc_ar_close"], rep
    assert rep["halo_pull"] == pr["chosen"].startswith("pull") and rep["halo_transport"] in ("in-kernel", "rccl")
    assert abs(rep["rnorm"] - one["rnorm"]) <= 1e-12 * one["rnorm"]


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


def test_cli_and_extension_share_one_rccl(mcg):
    """Both entry points run the same RCCL: the native CLI (thread per GPU) links the copies torch
    ships through build/rt, and the Python extension binds to them because torch is imported first.
    Same ncclGetVersion, same shared object."""
    info = mcg.native().rccl_info()
    assert info["version"] >= 22600, info
    p = _run([mcg.cli_path(), "--problem", "poisson2d", "--n", "32", "--force-comm", "--report", "json"])
    assert p.returncode == 0, p.stdout + p.stderr
    rep = json.loads(p.stdout.splitlines()[-2])
    assert rep["rccl_version"] == info["version"], (rep, info)
    assert os.path.realpath(rep["rccl_library"]) == os.path.realpath(info["library"]), (rep, info)


@pytest.mark.parametrize("route", ["spawn", "torchrun"])
@pytest.mark.parametrize("world", [2, 4])
def test_bench_multiprocess_rehearsal_on_one_gpu(route, world):
    """The P-rank bench's host side on ONE GPU, every round: P processes (bench.py's own launcher,
    or torchrun) on device 0 with collectives that move nothing, but the real gloo rendezvous,
    barriers, all_gather_object aggregation and slowest-rank JSON line of the scaling runs."""
    args = ["bench.py", "--gpus", str(world), "--rehearse-ranks", "--grid", "1024", "--steps", "10", "--warmup", "2",
            "--phases", "0", "--watchdog", "60"]
    if route == "spawn":
        cmd = [sys.executable] + args
    else:
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    p = _run(cmd, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["check"]["ok"] and line["steps"] == 10
    assert line["config"]["launch"] == route and line["config"]["parallelism"] == f"rehearse-rowpart{world}-one-gpu"
    assert line["check"]["device_iterations"] == 12 and line["check"]["rccl"]["version"] > 0


@pytest.mark.parametrize("mode", ["dual", "single"])
def test_one_rank_comm_modes_bitwise_equal_to_no_comm(mcg, mode):
    """The 1-rank RCCL communicator in both modes (two communicators, or one with every collective
    in one stream order) leaves the solve bitwise equal to the communicator-free one."""
    spec = mcg.make_problem("poisson2d", n=128, rhs="random")
    ref = mcg.CGSolver(spec, format="sellc8", recurrence=1).solve()
    s = mcg.CGSolver(spec, format="sellc8", recurrence=1, force_comm=True, comm_mode=mode)
    assert s.comm.serialized == (mode == "single")
    out = s.solve()
    assert out["iterations"] == ref["iterations"] and out["rnorm"] == ref["rnorm"]
    np.testing.assert_array_equal(out["x_local"], ref["x_local"])


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
