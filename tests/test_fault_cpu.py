"""Fault-handling threading contract (CPU, no GPU needed).

The heartbeat watchdog runs on a background thread.  It may only FLAG a dead peer (and set
the xGMI abort word); every teardown - ncclCommAbort, process-group destruction - must
happen on the main thread, which notices the flag between graph replays / steps
(``engine.poll``) and in its interruptible device waits, raises ``CommError`` and runs
``Trainer._recover``.  The epoch-end vote turns a failed xGMI wait on ONE rank into a
``CommError`` on every rank.
"""
import os
import threading
import time

import numpy as np
import pytest
import torch.distributed as dist

from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.parallel import CommError, Communicator, DistEnv
from distributed_neural_network_amd.parallel.fault import Heartbeat
from distributed_neural_network_amd.runtime import CpuEngine

from test_distributed_cpu import ROOT, _launch


def _comm_on(store_port: int) -> Communicator:
    c = Communicator(DistEnv(0, 1, 0, "127.0.0.1", store_port), "cpu")
    c.members = [0, 1]  # pretend to be rank 0 of a 2-rank group whose rank 1 never beats
    c.backend = "nccl"
    return c


def test_watchdog_flags_only_and_main_thread_raises():
    store = dist.TCPStore("127.0.0.1", 0, 1, is_master=True, wait_for_workers=False)
    comm = _comm_on(store.port)
    calls = {"abort": [], "signal": []}
    comm.abort = lambda: calls["abort"].append(threading.current_thread().name)
    real_signal = comm.signal_lost
    comm.signal_lost = lambda: (calls["signal"].append(threading.current_thread().name), real_signal())
    hb = Heartbeat(comm, period_s=0.05, timeout_s=0.3)
    try:
        t0 = time.time()
        while 1 not in hb.dead and time.time() - t0 < 10:
            time.sleep(0.02)
        assert 1 in hb.dead
        assert calls["abort"] == []                 # the thread never tears anything down
        assert calls["signal"] == ["dnn-heartbeat"]  # it only signals (xGMI abort word)
        assert comm.lost() == [1]
        with pytest.raises(CommError, match=r"\[1\] lost"):
            comm.check_alive()
    finally:
        hb.stop()


def test_engine_poll_aborts_mid_epoch():
    """A loss flagged mid-epoch stops the step loop at the next poll: no further step is
    issued behind a collective that cannot complete."""
    store = dist.TCPStore("127.0.0.1", 0, 1, is_master=True, wait_for_workers=False)
    comm = _comm_on(store.port)
    lost = []
    comm.watch = lambda: tuple(lost)
    eng = CpuEngine(batch=8, arena=init_arena(seed=0))
    eng.attach(synthetic(64, 0))
    eng.begin_epoch(np.arange(64, dtype=np.int32))
    eng.poll = comm.check_alive
    eng.run_steps(3)
    assert eng.epoch_stats(reset=False).batches == 3
    lost.append(1)  # the watchdog flags rank 1
    with pytest.raises(CommError):
        eng.run_steps(5)
    assert eng.epoch_stats(reset=False).batches == 3


def test_failed_wait_vote_raises_on_every_rank(tmp_path):
    r = _launch(2, [os.path.join(ROOT, "tests", "dist_worker.py"), "failvote", str(tmp_path), "0", "0", "0"],
                tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    for rank in (0, 1):
        msg = (tmp_path / f"vote{rank}.txt").read_text()
        assert "rank(s) [1]" in msg, (rank, msg)
