"""Process-group environment: who am I, how many of us, where is the rendezvous.

Capability parity: the reference gets rank/size from ``MPI.COMM_WORLD``
(data_parallelism_train.py:60-62) under ``mpiexec -n N`` (README.md:28).  Here a job
is one process per GPU; rank/size are read from the launcher's environment:
torchrun (RANK/WORLD_SIZE/LOCAL_RANK), OpenMPI (OMPI_COMM_WORLD_*), MPICH/Hydra and
Intel MPI (PMI_RANK/PMI_SIZE, MPI_LOCALRANKID), or Slurm (SLURM_PROCID/NTASKS) - so
``mpiexec -n 4 python data_parallelism_train.py`` still works without mpi4py.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


def _first(*names: str) -> str | None:
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return v
    return None


@dataclass(frozen=True)
class DistEnv:
    rank: int
    world: int
    local_rank: int
    master_addr: str
    master_port: int

    @property
    def distributed(self) -> bool:
        return self.world > 1


def detect() -> DistEnv:
    rank = _first("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", "SLURM_PROCID")
    world = _first("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS")
    local = _first("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "SLURM_LOCALID")
    r = int(rank) if rank is not None else 0
    w = int(world) if world is not None else 1
    lr = int(local) if local is not None else r
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    if not (0 <= r < w):
        raise ValueError(f"inconsistent rank {r} / world size {w} in the environment")
    return DistEnv(r, w, lr, addr, port)
