"""Both entry points accept every flag of the shared table (cuda_mpi_parallel_amd/cli_spec.py)
with the same value forms, and agree on the reference's default behaviour (CUDACG.cu:41-366)."""
import json
import subprocess

import pytest

from cuda_mpi_parallel_amd import __main__ as pycli
from cuda_mpi_parallel_amd.cli_spec import FLAGS

FILE_FLAGS = {"--matrix", "--rhs-file", "--checkpoint", "--resume"}


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("cli")
    m = d / "demo.mtx"
    m.write_text("%%MatrixMarket matrix coordinate real general\n3 3 5\n1 1 3\n1 3 2\n2 2 2\n3 1 2\n3 3 1\n")
    b = d / "b.txt"
    b.write_text("3.5\n1.5\n2.0\n")
    return {"--matrix": str(m), "--rhs-file": str(b), "--checkpoint": str(d / "ck"), "--resume": str(d / "ck")}


def _argv(flag, example, files):
    if flag in FILE_FLAGS:
        argv = [flag, files[flag]]
        if flag == "--rhs-file":
            argv = ["--matrix", files["--matrix"]] + argv
        return argv
    return [flag] if example is None else [flag, example]


@pytest.mark.parametrize("flag,example", [(f, e) for f, e, _ in FLAGS])
def test_both_clis_accept_flag(mcg, files, capsys, flag, example):
    argv = ["--device", "cpu"] + _argv(flag, example, files)
    p = subprocess.run([mcg.cli_path()] + argv, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, (argv, p.stdout, p.stderr)
    assert p.stdout.endswith("Success\n")
    rc = pycli.main(argv)
    out = capsys.readouterr().out
    assert rc == 0, (argv, out)
    assert out.endswith("Success\n")
    if flag not in ("--report", "--print-x"):
        assert out == p.stdout  # same x lines and the same final line


def test_unknown_flag_fails_in_both(mcg, capsys):
    p = subprocess.run([mcg.cli_path(), "--no-such-flag"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and p.stdout.startswith("invalid arguments")
    with pytest.raises(SystemExit) as e:
        pycli.main(["--no-such-flag"])
    assert e.value.code != 0


def test_json_reports_share_keys(mcg, capsys):
    argv = ["--device", "cpu", "--problem", "poisson2d", "--n", "16", "--report", "json"]
    p = subprocess.run([mcg.cli_path()] + argv, capture_output=True, text=True, timeout=60)
    native = json.loads(p.stdout.splitlines()[-2])
    assert pycli.main(argv) == 0
    py = json.loads(capsys.readouterr().out.splitlines()[-2])
    for k in ("problem", "n", "ranks", "device", "iterations", "converged", "breakdown", "rnorm", "solve_s",
              "it_per_s"):
        assert k in native and k in py
    assert native["iterations"] == py["iterations"] and native["n"] == py["n"] == 256
