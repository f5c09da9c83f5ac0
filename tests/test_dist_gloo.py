"""Multi-process CPU rehearsal of the distributed solver: world_size 2/3/4 processes over
torch.distributed (gloo, 127.0.0.1), each owning its rows with the GPU solver's halo plan."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, problem, kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import cuda_mpi_parallel_amd as mcg
    from cuda_mpi_parallel_amd.parallel.cpu_ref import cpu_cg_distributed, gather_x

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec = mcg.make_problem(problem, **kw)
        out = cpu_cg_distributed(spec, maxit=2000, tol=1e-7)
        x = gather_x(out)
        if rank == 0:
            q.put((out["iterations"], out["converged"], x))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("problem,kw", [("poisson2d", dict(n=40)), ("poisson3d", dict(n=10)),
                                         ("randspd", dict(rows=3000, band=20, density=0.3))])
def test_gloo_distributed_matches_single_process(mcg, C, world, problem, kw):
    spec = mcg.make_problem(problem, **kw)
    ref = C.cpu_cg(spec.native(), C.CgOptions(maxit=2000, tol=1e-7))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, problem, kw, q)) for r in range(world)]
    for p in procs:
        p.start()
    its, conv, x = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert abs(its - ref["iterations"]) <= 1 and conv == ref["converged"]
    np.testing.assert_allclose(x, ref["x"], rtol=1e-7, atol=1e-9 * (1 + np.abs(ref["x"]).max()))
