"""Process-per-GPU launcher (cuda_mpi_parallel_amd/parallel/launch.py) and bench.py's
job-level aggregation.  CPU only: the children here are plain Python scripts."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cuda_mpi_parallel_amd.parallel import launch  # noqa: E402


def test_child_env_is_torchrun_shaped():
    env = launch.child_env(3, 8, 29511, base={"PATH": "/bin"})
    assert env["RANK"] == "3" and env["LOCAL_RANK"] == "3"
    assert env["WORLD_SIZE"] == "8" and env["LOCAL_WORLD_SIZE"] == "8"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29511"
    assert env[launch.CHILD_FLAG] == "1"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert env["PATH"] == "/bin"


def _script(tmp_path, body):
    p = tmp_path / "child.py"
    p.write_text("import json, os, sys, time\n" + body)
    return str(p)


def test_spawn_ranks_env_and_rank0_stdout(tmp_path, capfd):
    out = tmp_path / "ranks"
    out.mkdir()
    s = _script(tmp_path, f"""
r = int(os.environ['RANK'])
keys = ['RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT', '{launch.CHILD_FLAG}']
open(os.path.join({str(out)!r}, str(r)), 'w').write(json.dumps({{k: os.environ[k] for k in keys}}))
print(json.dumps({{'rank': r, 'argv': sys.argv[1:]}}))
""")
    rc = launch.spawn_ranks(3, ["--x", "1"], script=s)
    assert rc == 0
    envs = [json.loads((out / str(r)).read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    lines = [json.loads(l) for l in capfd.readouterr().out.splitlines() if l.startswith("{")]
    assert lines == [{"rank": 0, "argv": ["--x", "1"]}]  # only rank 0 reaches stdout


def test_failing_rank_stops_the_others(tmp_path):
    s = _script(tmp_path, """
if os.environ['RANK'] == '1':
    sys.exit(3)
time.sleep(120)
""")
    t0 = time.monotonic()
    rc = launch.spawn_ranks(2, [], script=s, grace=5.0)
    assert rc == 3
    assert time.monotonic() - t0 < 30


def test_launch_or_none_inside_a_rank(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert launch.launch_or_none(None, []) is None
    assert launch.launch_or_none(2, []) is None
    assert launch.launch_or_none(4, []) == 2  # --gpus disagrees with the launcher's world


def test_launch_or_none_single_gpu_runs_inline(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert launch.launch_or_none(None, []) is None
    assert launch.launch_or_none(1, []) is None


def test_bench_too_many_gpus_fails_fast():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = "0"
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert p.stdout == ""
    assert len(p.stderr.strip().splitlines()) == 1 and "--gpus 2" in p.stderr
    assert time.monotonic() - t0 < 60


def test_bench_aggregate_takes_slowest_rank():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    ranks = [{"dt": 1.0, "ok": True, "iterations": 30}, {"dt": 2.0, "ok": True, "iterations": 30}]
    value, dt, ok = bench.aggregate(100, ranks)
    assert dt == 2.0 and value == pytest.approx(50.0) and ok
    ranks[1]["iterations"] = 31  # a rank latched at a different count: not ok
    assert not bench.aggregate(100, ranks)[2]
    ranks[1]["iterations"] = 30
    ranks[0]["ok"] = False
    assert not bench.aggregate(100, ranks)[2]


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    return bench


def test_bench_pass_labels():
    """The JSON names the pass the solver chose: plane carry for 3-D, the
    pipelined form with its replacement period, the split pass, the generic pass."""
    bench = _bench_module()
    carry3 = {"carry": True, "p3": True, "ap_recompute": True, "ar3_kw": 16}
    assert bench.pass_label(carry3, "poisson3d").startswith("plane-carry, three-term")
    assert bench.pass_label(dict(carry3, ar3_kw=0), "poisson2d").startswith("line-carry")
    assert bench.pass_label({"recurrence": "pipelined", "pipe_rr": 25}, "poisson2d") == (
        "pipelined CG (Ghysels-Vanroose: all-reduce || SpMV), residual replacement every 25")
    assert bench.pass_label({"recurrence": "pipelined", "pipe_rr": 0}, "randspd").startswith("pipelined CG")
    assert bench.pass_label({"pmat": True}, "randspd") == "split (materialized p)"
    assert bench.pass_label({}, "randspd") == "generic"
    # the lean-only kernels (uniform slice patterns) are named; the generic three-term ones are not
    assert bench.pass_label(dict(carry3, lean_only=True), "poisson3d").endswith(
        "lean runs (values in scalar registers, no codes streamed)")
    assert "lean" not in bench.pass_label(dict(carry3, lean_only=False), "poisson3d")


def test_kfd_gpu_count_from_a_fake_topology(tmp_path):
    """The launcher counts GPUs without HIP: KFD topology nodes with a nonzero gfx_target_version
    whose render node this process can open (a container sees the host's topology, not its cards)."""
    from cuda_mpi_parallel_amd.parallel import launch

    nodes, dri = tmp_path / "nodes", tmp_path / "dri"
    nodes.mkdir()
    dri.mkdir()
    specs = [(0, None), (90500, 128), (90500, 136), (90500, 144)]  # a CPU node and three GPUs
    for i, (gfx, minor) in enumerate(specs):
        d = nodes / str(i)
        d.mkdir()
        text = f"cpu_cores_count 8\ngfx_target_version {gfx}\n"
        if minor is not None:
            text += f"drm_render_minor {minor}\n"
        (d / "properties").write_text(text)
    for minor in (128, 144):  # only two of the three render nodes are in this "container"
        (dri / f"renderD{minor}").write_text("")
    assert launch.kfd_gpu_count(str(nodes), str(dri)) == 2
    assert launch.kfd_gpu_count(str(tmp_path / "missing"), str(dri)) is None
