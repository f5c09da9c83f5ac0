"""Process-per-GPU launcher: ``--gpus N`` without torchrun.

The reference pins one device (``cudaSetDevice(0)``, CUDACG.cu:87); here rank i drives
device i and the ranks talk over RCCL.  ``python bench.py --gpus N`` (and
``python -m cuda_mpi_parallel_amd --gpus N``) start N child processes of the same
script with the torchrun environment (RANK / WORLD_SIZE / LOCAL_RANK /
LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), so a rank runs the exact code
it runs under ``torch.distributed.run``.

The launcher itself never touches the GPU: it is called before the native extension
is loaded, counts devices without initialising HIP, and only forks/execs children
(it never ``exec``s itself).  A child that fails takes the others down (SIGTERM,
then SIGKILL after a grace period) so a rank stuck in a collective whose peer died
cannot hang the job; the launcher exits with the first failing child's status.

Only the standard library is used here: GPUs are counted the way the ROCm runtime enumerates
them -- KFD topology nodes in sysfs (``/sys/class/kfd/kfd/topology/nodes/*/properties``) with a
nonzero ``gfx_target_version`` whose render node ``/dev/dri/renderD<drm_render_minor>`` this
process can open (a container sees the host's whole topology but only its own render nodes) --
and the ``*_VISIBLE_DEVICES`` variables, so the parent cannot initialise HIP before it forks
the ranks; ``torch.cuda.device_count()`` is only the fallback when there is no KFD topology.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence

CHILD_FLAG = "MCG_LAUNCHED_RANK"


def under_launcher() -> bool:
    """True inside a rank started by torchrun or by :func:`spawn_ranks`."""
    return "WORLD_SIZE" in os.environ


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def kfd_gpu_count(root: str = KFD_NODES, dri: str = "/dev/dri") -> Optional[int]:
    """GPUs this process can open: KFD topology nodes with a nonzero gfx_target_version whose
    render node is accessible; None without a KFD topology."""
    try:
        nodes = os.listdir(root)
    except OSError:
        return None
    n = 0
    for node in nodes:
        props = {}
        try:
            with open(os.path.join(root, node, "properties")) as f:
                for line in f:
                    k, _, v = line.strip().partition(" ")
                    props[k] = v.strip()
            if int(props.get("gfx_target_version", "0") or "0") == 0:
                continue
            minor = props.get("drm_render_minor")
            if minor is not None and not os.access(os.path.join(dri, f"renderD{int(minor)}"), os.R_OK | os.W_OK):
                continue
            n += 1
        except (OSError, ValueError):
            continue
    return n


def visible_devices() -> int:
    """Number of GPUs this process may use (no HIP initialisation)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip() != "":
            n_env = len([t for t in v.split(",") if t.strip() != ""])
            break
    else:
        n_env = None
    n = kfd_gpu_count()
    if n is None:  # no KFD topology (not a ROCm host): ask torch, which does not initialise HIP either
        try:
            import warnings

            import torch

            with warnings.catch_warnings():  # torch warns when amdsmi finds no GPU (CPU hosts)
                warnings.simplefilter("ignore")
                n = int(torch.cuda.device_count())
        except Exception:  # pragma: no cover - torch missing / broken
            n = 0
    return n if n_env is None else min(n, n_env)


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return int(s.getsockname()[1])


def child_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """Environment of rank ``rank``: the variables torchrun would set (single node)."""
    env = dict(os.environ if base is None else base)
    env.update({
        "RANK": str(rank),
        "LOCAL_RANK": str(rank),
        "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(world),
        "GROUP_RANK": "0",
        "MASTER_ADDR": "127.0.0.1",
        "MASTER_PORT": str(port),
        CHILD_FLAG: "1",
    })
    # the host driver only supports dmabuf IPC: RCCL / tensor sharing need this (see README)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _stop(procs: Sequence[subprocess.Popen], grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                p.send_signal(signal.SIGTERM)
            except ProcessLookupError:  # pragma: no cover
                pass
    t_end = time.monotonic() + grace
    for p in procs:
        left = max(0.0, t_end - time.monotonic())
        try:
            p.wait(timeout=left)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def spawn_ranks(world: int, argv: List[str], script: Optional[str] = None, module: Optional[str] = None,
                grace: float = 10.0, quiet_nonzero_stdout: bool = True) -> int:
    """Run ``python <script> <argv>`` (or ``python -m <module> <argv>``) as ``world`` ranks;
    return the job's exit status.

    Rank 0 keeps stdout (it prints the result line); other ranks' stdout is dropped when
    ``quiet_nonzero_stdout``.  stderr of every rank is inherited.
    """
    if world < 1:
        print(f"launcher: invalid number of ranks {world}", file=sys.stderr)
        return 2
    head = ["-m", module] if module else [script or os.path.abspath(sys.argv[0])]
    cmd = [sys.executable] + head + list(argv)
    port = free_port()
    procs: List[subprocess.Popen] = []
    try:
        for r in range(world):
            out = subprocess.DEVNULL if (quiet_nonzero_stdout and r > 0) else None
            procs.append(subprocess.Popen(cmd, env=child_env(r, world, port), stdout=out))
        status = 0
        while True:
            alive = 0
            for p in procs:
                rc = p.poll()
                if rc is None:
                    alive += 1
                elif rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"launcher: rank {procs.index(p)} exited with status {rc}; stopping the other ranks",
                          file=sys.stderr)
                    _stop(procs, grace)
            if status != 0 or alive == 0:
                break
            time.sleep(0.05)
        return status
    except BaseException:
        _stop(procs, grace)
        raise


def launch_or_none(gpus: Optional[int], argv: List[str], force_spawn: bool = False,
                   script: Optional[str] = None, module: Optional[str] = None,
                   share_device: bool = False) -> Optional[int]:
    """Entry-point helper.  Returns None when this process should run as a rank itself
    (already under a launcher, or a single GPU without ``force_spawn``); otherwise checks
    the device count, starts the ranks and returns the job's exit status.

    ``share_device``: the ranks may outnumber the GPUs (a rehearsal whose ranks share device 0
    and move no data between GPUs); the device-count check is skipped."""
    if under_launcher():
        world = int(os.environ["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            print(f"launcher: --gpus {gpus} but WORLD_SIZE={world}", file=sys.stderr)
            return 2
        return None
    n = 1 if gpus is None else gpus
    if n == 1 and not force_spawn:
        return None
    have = n if share_device else visible_devices()
    if n > have:
        print(f"launcher: --gpus {n} but {have} GPU(s) visible", file=sys.stderr)
        return 2
    return spawn_ranks(n, argv, script=script, module=module)
