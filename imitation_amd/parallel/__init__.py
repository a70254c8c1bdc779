"""Distributed (data-parallel) layer over RCCL/xGMI; see :mod:`imitation_amd.parallel.dist`."""

from imitation_amd.parallel import dist
from imitation_amd.parallel.dist import (
    GradBucket,
    all_gather_rows,
    allreduce_grads,
    allreduce_scalars,
    barrier,
    broadcast_module,
    init,
    is_main,
    rank,
    world_size,
)

__all__ = [
    "dist",
    "GradBucket",
    "all_gather_rows",
    "allreduce_grads",
    "allreduce_scalars",
    "barrier",
    "broadcast_module",
    "init",
    "is_main",
    "rank",
    "world_size",
]
