"""Distribution layer: 1-D row partition, halo plans, RCCL bootstrap, CPU gloo reference.

The reference has no distribution at all (single ``cudaSetDevice(0)``,
CUDACG.cu:87).  The north star (BASELINE.json:5) row-partitions the matrix over the
GPUs of one node, all-reduces the two CG dot products and exchanges boundary rows.
"""
from .plan import Layout, layout, partition_rows  # noqa: F401
from .dist import (  # noqa: F401
    DistEnv,
    bootstrap_comm,
    dist_env,
    init_process_group,
)
from .cpu_ref import cpu_cg_distributed  # noqa: F401

__all__ = [
    "Layout",
    "layout",
    "partition_rows",
    "DistEnv",
    "dist_env",
    "init_process_group",
    "bootstrap_comm",
    "cpu_cg_distributed",
]
