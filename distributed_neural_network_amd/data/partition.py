"""Dataset partitioning and per-epoch sample orders.

Capability parity: ``partition_dataset`` (data_parallelism_train.py:49-53) gives
worker ``rank in [1, size)`` the contiguous slice ``[(rank-1)*ps, rank*ps)`` with
``ps = len // (size-1)`` and drops the remainder; ``DataLoader(shuffle=True)``
(data_parallelism_train.py:74-79) reshuffles that slice every epoch.  Model
replication (model_replication_train.py:40-45) gives every worker the full set.

Here a rank's epoch is an int32 list of sample ids (uploaded to HBM, read by the
fused kernel), drawn by the native seeded Fisher-Yates so that a given
(seed, epoch, rank) produces the same order on CPU and GPU.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..ops import native


def shard_bounds(n: int, rank: int, world: int, parent: bool = False) -> tuple[int, int]:
    """Contiguous shard of ``n`` samples for ``rank``.

    ``parent=True`` is the reference layout (rank 0 is a non-training parameter
    server, workers are ranks 1..world-1); otherwise every rank trains.
    """
    if parent:
        if world < 2:
            raise ValueError("parent/child layout needs at least 2 processes (rank 0 does not train)")
        if rank == 0:
            return 0, 0
        ps = n // (world - 1)
        return (rank - 1) * ps, rank * ps
    ps = n // world
    return rank * ps, (rank + 1) * ps


@dataclass
class EpochSampler:
    """Sample ids of one rank's epoch: a shard (or the whole set) reshuffled per epoch."""

    indices: np.ndarray   # int32 sample ids this rank owns
    seed: int
    stream: int           # per-rank stream id (replication: different shuffles per rank)
    shuffle: bool = True

    @classmethod
    def for_rank(cls, n: int, rank: int, world: int, seed: int, mode: str = "shard",
                 parent: bool = False, shuffle: bool = True) -> "EpochSampler":
        if mode == "shard":
            lo, hi = shard_bounds(n, rank, world, parent)
            idx = np.arange(lo, hi, dtype=np.int32)
        elif mode == "full":
            idx = np.arange(n, dtype=np.int32)
        else:
            raise ValueError(f"unknown partition mode {mode!r}")
        return cls(idx, seed, rank, shuffle)

    def __len__(self) -> int:
        return int(self.indices.shape[0])

    def order(self, epoch: int) -> np.ndarray:
        if not self.shuffle or len(self) == 0:
            return self.indices.copy()
        return native.io().shuffled(self.indices, self.seed, epoch, self.stream)

    def steps(self, batch: int) -> int:
        """Batches per epoch with drop_last=False (DataLoader default)."""
        return (len(self) + batch - 1) // batch
