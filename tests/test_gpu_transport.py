"""P > 1 transports at both entry points, rehearsed on ONE GPU.

``bin/mcg-cg --gpus P --rehearse-ranks`` runs its P rank threads on GPU 0 with the in-process
communicator (LocalComm) wrapped exactly as at P GPUs: a PeerHaloComm that maps the other threads'
halo buffers as plain pointers, so the lean carries read their ghost lines in-kernel (halo_pull), and
the solver's transport probe times the pulled against the exchanged halo at the first reset.
``python -m cuda_mpi_parallel_amd --gpus P --rehearse-ranks`` runs P processes on GPU 0 with the IPC
all-reduce and the peer-mapped halo (the real P-rank recurrence across processes).  Both must
reproduce the one-rank solve.  Reference: the reductions CUDACG.cu:304,328 and the neighbour reads of
the SpMV, :288, which these transports carry; the entry point, :41.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, timeout=300):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


def _report(p):
    assert p.returncode == 0, p.stdout + p.stderr
    return json.loads(p.stdout.splitlines()[-2])


FIXED = ["--fixed-iters", "40", "--report", "json", "--print-x", "no", "--watchdog", "120"]


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("problem", [["--problem", "poisson2d", "--n", "2048"], ["--problem", "poisson3d", "--n", "128"]])
def test_native_cli_rehearsed_ranks_pull_and_match_one_rank(mcg, world, problem):
    if world == 8 and problem[1] == "poisson2d":
        problem = ["--problem", "poisson2d", "--n", "4096"]  # 512 lines a rank (256 are too few for the lean runs)
    one = _report(_run([mcg.cli_path()] + problem + FIXED))
    rep = _report(_run([mcg.cli_path(), "--gpus", str(world), "--rehearse-ranks"] + problem + FIXED))
    assert rep["ranks"] == world and rep["rehearse_ranks"]
    pr = rep["transport_probe"]
    if pr is None:  # the pull was no candidate (a 3-D rank of 16 planes may be too short for the lean runs)
        assert problem[1] == "poisson3d" and world == 8 and not rep["halo_pull"], rep
        assert abs(rep["rnorm"] - one["rnorm"]) <= 1e-13 * one["rnorm"]
        return
    # the probe ran both halo arms on the mapped buffers and the pulled run reproduced the exchanged one
    assert pr is not None and pr["pull_bitwise"] and pr["pull_us"] > 0 and pr["rccl_halo_us"] > 0, rep
    assert rep["halo_pull"] == (pr["pull_us"] <= pr["rccl_halo_us"]) == pr["chosen"].startswith("pull"), rep
    assert rep["halo_transport"] == ("in-kernel" if rep["halo_pull"] else "local")
    assert rep["iterations"] == one["iterations"] == 40
    assert abs(rep["rnorm"] - one["rnorm"]) <= 1e-13 * one["rnorm"], (rep["rnorm"], one["rnorm"])


def test_native_cli_rehearsed_ranks_probe_off_keeps_the_pull(mcg):
    """--transport-probe off: the configured default (the pull, verified at the first reset) runs."""
    problem = ["--problem", "poisson2d", "--n", "2048"]
    one = _report(_run([mcg.cli_path()] + problem + FIXED))
    rep = _report(_run([mcg.cli_path(), "--gpus", "4", "--rehearse-ranks", "--transport-probe", "off"] + problem + FIXED))
    assert rep["halo_pull"] and rep["transport_probe"] is None and rep["halo_transport"] == "in-kernel"
    assert abs(rep["rnorm"] - one["rnorm"]) <= 1e-13 * one["rnorm"]
    rep = _report(_run([mcg.cli_path(), "--gpus", "4", "--rehearse-ranks", "--halo-transport", "rccl"] + problem + FIXED))
    assert not rep["halo_pull"] and rep["transport_probe"] is None
    assert abs(rep["rnorm"] - one["rnorm"]) <= 1e-13 * one["rnorm"]


def test_python_cli_rehearsed_ranks_match_one_rank(mcg):
    problem = ["--problem", "poisson2d", "--n", "2048"]
    one = _report(_run([sys.executable, "-m", "cuda_mpi_parallel_amd"] + problem + FIXED))
    rep = _report(_run([sys.executable, "-m", "cuda_mpi_parallel_amd", "--gpus", "2", "--rehearse-ranks"]
                       + problem + FIXED))
    assert rep["ranks"] == 2 and rep["rehearse_ranks"] and rep["allreduce"] == "ipc"
    pr = rep["transport_probe"]
    assert pr is not None and pr["pull_bitwise"], rep
    assert rep["halo_pull"] == pr["chosen"].startswith("pull")
    assert abs(rep["rnorm"] - one["rnorm"]) <= 1e-13 * one["rnorm"], (rep["rnorm"], one["rnorm"])
