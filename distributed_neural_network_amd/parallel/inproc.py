"""In-process N-rank harness of the per-step xGMI exchange: N engines, ONE process, ONE GPU, one
stream each - no IPC, no process group, no time-slicing.

Why: every multi-rank GPU measurement so far ran two PROCESSES on one GPU.
Their persistent grids are time-sliced by the scheduler, so the in-launch exchange waited out
the other process' slice (exchange wait p99 54 us) and the ``-pers`` forms lost 77 vs 51 us to
the serial exchange on a setup that says nothing about distinct GPUs.  Here the "ranks" are N
``HipEngine``s of one process, each launching on its own HIP stream; their grids run
concurrently on disjoint CUs (2 x (57 + 64) = 242 of the 248 resident workgroups at batch 64).
Every rank's exchange region is ordinary uncached device memory of this process (the same
allocation the IPC path exports), addressed directly by the peers - the kernels run the exact
protocol, code and instances of the multi-GPU path; only the link is the local memory instead of
xGMI.  So the harness measures the protocol's own cost (the waits between the two grids, the
extra work in the reduction workgroups) and pins its result bit for bit to the serial one-launch
exchange.

Used by ``tools/inproc_pair.py`` (timings -> JSON) and ``tests/test_inproc_pair_gpu.py``.
Reference parity: the per-step gradient all-reduce is the report's future work
(Project_Report.pdf p.4 §6.2) over the reference's training loop
(data_parallelism_train.py:193-213, averaging :238-240).
"""
from __future__ import annotations

import time
from types import SimpleNamespace

import numpy as np
import torch

from ..models.network import LAYOUT
from .xgmi import EXCHANGE_MODES, XgmiGradSync, XgmiGroup


class InprocGroup(XgmiGroup):
    """One rank's view of an in-process exchange group: the same launch state as an
    ``XgmiGroup`` (step counters, sticky error word, abort word, wait ring), with the peers'
    regions addressed directly instead of through IPC handles."""

    def __init__(self, ext, device: torch.device, rank: int, world: int, capacity: int,
                 timeout_s: float = 5.0) -> None:
        self.comm = SimpleNamespace(device=device, watch=None, rank=rank, world=world, generation=0)
        self.ext = ext
        self.capacity = int(capacity)
        self.timeout_s = float(timeout_s)
        self.rank, self.world, self.generation = rank, world, 0
        self.opened: list[int] = []
        self.abort_host, self.abort_dev = ext.xgmi_abort_word()
        with torch.cuda.device(device):
            self.local, _handle, self.kind = ext.xgmi_alloc(self.capacity)
        nb = ext.xgmi_max_blocks(self.capacity)
        self.ctr = torch.zeros(nb + 1, device=device, dtype=torch.int32)
        self.xp_ctr = torch.zeros(ext.xgmi_xp_max_blocks(), device=device, dtype=torch.int32)
        self.one_launch, self.broken, self.xp_mode, self.ar_mode = True, False, 0, 0
        self.wait = None
        self.regions: list[int] = []
        self.devices = 1


_OWN_QUEUE: dict = {}  # device index -> streams with a hardware queue of their own (never destroyed)


def own_queue_streams(engines: list) -> list:
    """One stream per rank, each with a HARDWARE queue of its own (a CU-masked stream over every
    CU: csrc/bindings.cpp stream_create_own_queue).  Ordinary streams share the process' few
    hardware queues (GPU_MAX_HW_QUEUES, 4): two ranks whose streams share one run one after the
    other, and a rank's exchange then waits for granules its peer cannot publish until the wait
    times out.  Which streams share a queue depends on every stream the process created before
    (tools/inproc_stream_probe.py: one extra stream created first was enough).  The streams are
    kept for the life of the process and handed out again: the caching allocator keeps blocks
    of tensors allocated on a stream tied to that stream, so it must never be destroyed."""
    dev = engines[0].device
    pool = _OWN_QUEUE.setdefault(dev.index if dev.index is not None else torch.cuda.current_device(), [])
    with torch.cuda.device(dev):
        while len(pool) < len(engines):
            pool.append(torch.cuda.ExternalStream(engines[0].ext.stream_create_own_queue(), device=dev))
    return pool[:len(engines)]


def release_streams(engines: list, streams: list) -> None:
    """The ranks' work is done (the streams stay in the pool for the next harness)."""
    torch.cuda.synchronize(engines[0].device)


def build_pair(engines: list, mode: int = 0, timeout_s: float = 5.0, record_waits: bool = True) -> list[InprocGroup]:
    """Install an in-process exchange group of form ``mode`` (xgmi.EXCHANGE_MODES: 0 pull, 2
    two-hop) on every engine of ``engines`` (one rank each, rank = list index)."""
    world = len(engines)
    if not 1 <= world <= 8:
        raise ValueError("1..8 in-process ranks")
    dev = engines[0].device
    groups = [InprocGroup(e.ext, dev, r, world, LAYOUT.total, timeout_s) for r, e in enumerate(engines)]
    regions = [g.local for g in groups]
    for g, e in zip(groups, engines):
        g.regions = list(regions)
        g.xp_mode = mode
        g.enable_wait_stats(record_waits)
        e.grad_sync = XgmiGradSync(g)
        e.pers_exchange = False
        e.invalidate_graphs()
    return groups


def set_form(engines: list, groups: list, form: str) -> None:
    """Switch every engine to ``form``: ``local`` (no exchange), ``xgmi-pull`` / ``xgmi-rsag``
    (the serial one-launch exchange) or ``xgmi-pull-pers`` / ``xgmi-rsag-pers`` (the exchange
    inside the persistent launch)."""
    for e, g in zip(engines, groups):
        e.invalidate_graphs()
        if form == "local":
            e.grad_sync = None
            e.pers_exchange = False
            continue
        g.xp_mode = EXCHANGE_MODES[form[len("xgmi-"):].removesuffix("-pers")]
        e.grad_sync = XgmiGradSync(g)
        e.pers_exchange = form.endswith("-pers")


def close(engines: list, groups: list) -> None:
    torch.cuda.synchronize(engines[0].device)
    for e in engines:
        e.grad_sync = None
        e.pers_exchange = False
        e.invalidate_graphs()
    for g in groups:
        g.close()


class PairRunner:
    """Drives N engines together: ``run(n)`` queues n steps on every engine's own stream (epoch
    boundaries included: each engine walks its own shard), ``window(n)`` times it like bench.py's
    window (device sync on both sides; wall clock and per-stream events)."""

    def __init__(self, engines: list, orders: list[np.ndarray]) -> None:
        self.engines, self.orders = engines, orders
        for e in engines:  # the engines' launches must be in flight together: no synchronous direct dispatch
            e.direct = False
        self.streams = own_queue_streams(engines)
        self.spe = engines[0].steps_per_epoch() if engines[0].order_len else None
        self.left = 0

    def release(self) -> None:
        release_streams(self.engines, self.streams)
        self.streams = []

    def begin(self) -> None:
        for e, s, o in zip(self.engines, self.streams, self.orders):
            with torch.cuda.stream(s):
                e.begin_epoch(o)
        self.spe = self.engines[0].steps_per_epoch()
        self.left = self.spe

    def prepare(self, steps: int) -> None:
        """Capture every chunk graph + the exact-size graph of ``steps`` (outside timing).  Every
        rank's graphs must exist before any rank replays one: a capture synchronizes the device,
        so capturing while a peer's replay waits on this rank's granules ends in a timed-out wait."""
        for e, s in zip(self.engines, self.streams):
            with torch.cuda.stream(s):
                e.prepare_graphs(exact=(steps,))

    def run(self, n: int) -> None:
        while n > 0:
            if self.left == 0:
                self.begin()
            k = min(n, self.left)
            for e, s in zip(self.engines, self.streams):
                with torch.cuda.stream(s):
                    e.run_steps(k)
            self.left -= k
            n -= k

    def window(self, steps: int) -> tuple[float, float]:
        """(wall us/step, max over streams of the event-timed us/step) of ``steps`` steps."""
        dev = self.engines[0].device
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in self.engines]
        t0 = time.perf_counter()
        for (a, _), s in zip(ev, self.streams):
            a.record(s)
        self.run(steps)
        for (_, b), s in zip(ev, self.streams):
            b.record(s)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        gpu = max(a.elapsed_time(b) for a, b in ev) * 1e-3
        return 1e6 * wall / steps, 1e6 * gpu / steps


__all__ = ["InprocGroup", "PairRunner", "build_pair", "close", "own_queue_streams", "release_streams", "set_form"]
