"""The mcg-cg binary: the reference's entry-point semantics (CUDACG.cu:41-366)."""
import json
import subprocess

import pytest


def run(mcg, *args, timeout=300):
    return subprocess.run([mcg.cli_path(), *args], capture_output=True, text=True, timeout=timeout)


def test_cpu_demo_golden_stdout(mcg):
    p = run(mcg, "--device", "cpu")
    assert p.returncode == 0
    assert p.stdout == "0.500000\n0.750000\n1.000000\nSuccess\n"


def test_virtual_ranks_cpu_demo(mcg):
    p = run(mcg, "--device", "cpu", "--sim-ranks", "2")
    assert p.returncode == 0 and p.stdout == "0.500000\n0.750000\n1.000000\nSuccess\n"


def test_bad_argument_prints_message_and_exits_1(mcg):
    p = run(mcg, "--problem", "nope")
    assert p.returncode == 1
    assert p.stdout.strip() == "unknown problem: nope"


def test_no_gpu_error_path(mcg):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = run(mcg)  # default = GPU 0; without a device: one message on stdout, exit 1 (CUDACG.cu:88-91)
    assert p.returncode == 1 and p.stdout == "Device Set failed\n"


def test_json_report_cpu_poisson(mcg):
    p = run(mcg, "--device", "cpu", "--problem", "poisson2d", "--n", "64", "--report", "json")
    assert p.returncode == 0
    lines = p.stdout.strip().splitlines()
    assert lines[-1] == "Success"
    rep = json.loads(lines[-2])
    assert rep["problem"] == "poisson2d" and rep["n"] == 4096 and rep["converged"]
    assert rep["rnorm"] < 1e-7
    assert rep["device_bytes_per_rank"] == []  # CPU path holds no device memory


def test_fixed_iterations_cpu(mcg):
    p = run(mcg, "--device", "cpu", "--problem", "poisson2d", "--n", "64", "--fixed-iters", "17", "--report", "json")
    rep = json.loads(p.stdout.strip().splitlines()[-2])
    assert rep["iterations"] == 17 and not rep["converged"]


def test_python_module_cli_cpu_golden(mcg):
    import sys

    p = subprocess.run([sys.executable, "-m", "cuda_mpi_parallel_amd", "--device", "cpu"], capture_output=True,
                       text=True, timeout=300, cwd=mcg.repo_root())
    assert p.returncode == 0 and p.stdout == "0.500000\n0.750000\n1.000000\nSuccess\n"
