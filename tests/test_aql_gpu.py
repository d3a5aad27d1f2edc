"""Direct AQL dispatch of the persistent launch (csrc/runtime/aql_dispatch.h, DNN_AQL=1): the
same kernel object through this process's own HSA queue must give the graph replays' bits."""
import numpy as np
import pytest
import torch

from distributed_neural_network_amd.data import synthetic
from distributed_neural_network_amd.models.network import init_arena
from distributed_neural_network_amd.runtime import HipEngine

pytestmark = pytest.mark.gpu


def _engine(arena, direct, dtype="bf16"):
    eng = HipEngine(batch=64, arena=arena, graph_chunk=8, dtype=dtype)
    if not eng.persist:
        pytest.skip("the persistent launch is off on this device")
    if direct:
        why = eng.ext.aql_status(torch.cuda.current_device())
        assert why == "", f"no AQL queue on a GPU box: {why}"
    eng.direct = direct  # (on by default: the reference side turns it off)
    return eng


def _run(eng, data, orders, steps):
    eng.attach(data)
    stats = []
    for order in orders:
        eng.begin_epoch(order)
        for n in steps:
            eng.run_steps(n)
        stats.append(eng.epoch_stats())
    torch.cuda.synchronize()
    return eng.master.cpu(), eng.mom.cpu(), eng.shadow.cpu(), stats


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_direct_dispatch_matches_graph_replays(dtype):
    """1-, 5- and 20-step launches, a tail batch, steps past an epoch's end, two epochs."""
    data = synthetic(1000, 4)  # 16 steps per epoch incl. a 40-sample tail
    a = init_arena(seed=5)
    rng = np.random.default_rng(1)
    orders = [rng.permutation(1000).astype(np.int32) for _ in range(2)]
    steps = (1, 5, 20)  # 26 steps: past the epoch's end (no-op steps)
    ref = _run(_engine(a, False, dtype), data, orders, steps)
    eng = _engine(a, True, dtype)
    got = _run(eng, data, orders, steps)
    assert eng._direct_h, "the direct path did not run"
    for x, y in zip(ref[:3], got[:3]):
        assert torch.equal(x, y)
    for s0, s1 in zip(ref[3], got[3]):
        assert s0.loss_sum == s1.loss_sum and s0.correct == s1.correct and s0.samples == s1.samples == 1000
    assert not eng.step_wait_failed()


def test_direct_dispatch_orders_after_stream_work():
    """A window queued right behind stream work (an epoch start, a parameter reload) must see it:
    the direct path waits for the stream before its dispatch."""
    data = synthetic(640, 6)
    a = init_arena(seed=7)
    order = np.arange(640, dtype=np.int32)
    res = []
    for direct in (False, True):
        eng = _engine(a, direct)
        eng.attach(data)
        eng.begin_epoch(order)
        eng.run_steps(3)
        eng.master.mul_(0.5)  # queued stream work the next window must see
        eng.params_changed()
        eng.run_steps(4)
        torch.cuda.synchronize()
        res.append(eng.master.cpu())
    assert torch.equal(res[0], res[1])


class _NoDirectExt:
    """The extension with a persistent launcher that refuses to prepare direct dispatches."""

    def __init__(self, ext):
        self._ext = ext

    def __getattr__(self, name):
        return getattr(self._ext, name)

    def fused_train_persist(self, *a, direct=False, **k):
        if direct:
            raise RuntimeError("injected: no direct dispatch")
        return self._ext.fused_train_persist(*a, **k)


def test_direct_dispatch_failure_falls_back_to_graphs():
    """A launch shape whose direct dispatch cannot be prepared runs as graph replays (same bits),
    and the engine says why."""
    data = synthetic(640, 8)
    a = init_arena(seed=9)
    order = np.arange(640, dtype=np.int32)
    ref = _run(_engine(a, False), data, [order], (3, 4))
    eng = _engine(a, True)
    eng.ext = _NoDirectExt(eng.ext)
    got = _run(eng, data, [order], (3, 4))
    assert not eng.direct and "injected" in eng.direct_why and not eng._direct_h
    assert torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])


def test_direct_dispatch_overlaps_host_work():
    """run_steps(n, host_work): the host work runs while the dispatched steps run (launch, work,
    wait), and the steps give the same bits."""
    data = synthetic(640, 3)
    a = init_arena(seed=4)
    order = np.arange(640, dtype=np.int32)
    res, calls = [], []
    for direct in (False, True):
        eng = _engine(a, direct)
        eng.attach(data)
        eng.begin_epoch(order)
        eng.run_steps(6, host_work=lambda: calls.append(direct))
        torch.cuda.synchronize()
        res.append(eng.master.cpu())
    assert calls == [False, True] and torch.equal(res[0], res[1])


def test_aql_selftest_passes():
    """The direct path end to end on a trivial kernel (host kernel arguments, dynamic LDS, more
    workgroups than CUs): what the engine runs once per device before its first direct launch."""
    ext = HipEngine(batch=64).ext
    assert ext.aql_selftest() == ""
