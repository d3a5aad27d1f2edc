"""Phase timers.

Capability parity: the reference's module-level accumulators
``data_loading_time``, ``training_time``, ``evaluation_time``,
``mpi_communication_time_parent`` and ``mpi_communication_time_children``
(data_parallelism_train.py:32-37, accumulated with time.time() deltas at :68-96,
:116-120, :136-139, :158-179, :190-213, :228-246).

Differences: a phase is closed with a device synchronise
when timing GPU work, so the number is the real device time of the phase; and the
time spent *waiting* inside collectives is measured as part of the communication
phase (the reference timed only the bookkeeping after recv returned).
"""
from __future__ import annotations

import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Callable, Dict, Optional

from . import roctx


class PhaseTimers:
    # names used by the reference log files
    DATA = "data_loading"
    TRAIN = "training"
    EVAL = "evaluation"
    COMM_PARENT = "comm_parent"
    COMM_CHILDREN = "comm_children"

    def __init__(self, sync: Optional[Callable[[], None]] = None) -> None:
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        self._sync = sync

    @contextmanager
    def phase(self, name: str, sync: bool = True):
        if sync and self._sync is not None:
            self._sync()
        roctx.push(name)
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync and self._sync is not None:
                self._sync()
            self.totals[name] += time.perf_counter() - t0
            self.counts[name] += 1
            roctx.pop()

    def add(self, name: str, seconds: float) -> None:
        self.totals[name] += seconds
        self.counts[name] += 1

    def __getitem__(self, name: str) -> float:
        return self.totals.get(name, 0.0)

    def as_dict(self) -> Dict[str, float]:
        return dict(self.totals)
