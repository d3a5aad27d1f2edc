"""EpochCursor: steps cross epoch boundaries without skipping any, and an engine whose run_steps
takes host work gets the next epoch's shuffle to overlap the steps that end the current one."""
import numpy as np

from distributed_neural_network_amd.runtime.cursor import EpochCursor


class _Sampler:
    def __init__(self):
        self.calls = []

    def steps(self, batch):
        return 3

    def order(self, epoch):
        self.calls.append(epoch)
        return np.arange(6) + 100 * epoch


class _Policy:
    def epoch_end(self, engine, epoch):
        engine.log.append(("end", epoch))

    def epoch_start(self, engine, epoch):
        engine.log.append(("start", epoch))


class _Engine:
    def __init__(self):
        self.log = []

    def begin_epoch(self, order):
        self.log.append(("begin", int(order[0])))


class _AheadEngine(_Engine):
    def run_steps(self, n, host_work=None):
        self.log.append(("run", n, host_work is not None))
        if host_work is not None:
            host_work()


class _PlainEngine(_Engine):
    def run_steps(self, n):
        self.log.append(("run", n))


def test_shuffle_ahead_overlaps_the_steps_that_end_an_epoch():
    c = EpochCursor(_AheadEngine(), _Sampler(), _Policy(), 2)
    c.run(7)
    assert c.engine.log == [("start", 0), ("begin", 0), ("run", 3, True), ("end", 0), ("start", 1), ("begin", 100),
                            ("run", 3, True), ("end", 1), ("start", 2), ("begin", 200), ("run", 1, False)]
    assert c.sampler.calls == [0, 1, 2]  # each epoch shuffled once, epochs 1 and 2 ahead of time
    c.run(2)  # the rest of epoch 2: nothing ahead
    assert c.engine.log[-1] == ("run", 2, False) and c.left == 0


def test_engines_without_host_work_run_as_before():
    c = EpochCursor(_PlainEngine(), _Sampler(), _Policy(), 2)
    c.run(7)
    assert [e for e in c.engine.log if e[0] == "run"] == [("run", 3), ("run", 3), ("run", 1)]
    assert c.sampler.calls == [0, 1, 2]
