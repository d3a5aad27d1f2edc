"""Step runner that crosses epoch boundaries (bench windows, the all-reduce A/B)."""
from __future__ import annotations

import inspect


class EpochCursor:
    """Feeds k optimizer steps to the engine, starting a new shuffled epoch (policy epoch_end /
    epoch_start + ``engine.begin_epoch``) whenever one ends - no step is skipped."""

    def __init__(self, engine, sampler, policy, batch: int) -> None:
        self.engine, self.sampler, self.policy, self.batch = engine, sampler, policy, batch
        self.epoch = -1
        self.left = 0
        self.steps_per_epoch = sampler.steps(batch)
        self._orders: dict[int, object] = {}  # epoch -> its order, shuffled ahead of time
        # engines whose run_steps can overlap host work with its steps (HipEngine's direct dispatch)
        self._ahead = "host_work" in inspect.signature(engine.run_steps).parameters

    def _order(self, epoch: int):
        o = self._orders.pop(epoch, None)
        return self.sampler.order(epoch) if o is None else o

    def _shuffle_ahead(self) -> None:
        """The next epoch's shuffle (host work), while the steps that end this one run."""
        self._orders[self.epoch + 1] = self.sampler.order(self.epoch + 1)

    def _next_epoch(self) -> None:
        if self.epoch >= 0:
            self.policy.epoch_end(self.engine, self.epoch)
        self.epoch += 1
        self.policy.epoch_start(self.engine, self.epoch)
        self.engine.begin_epoch(self._order(self.epoch))
        self.left = self.steps_per_epoch

    def run(self, k: int) -> None:
        while k > 0:
            if self.left == 0:
                self._next_epoch()
            n = min(k, self.left)
            if self._ahead and n < k and self.epoch + 1 not in self._orders:  # it goes on into the next epoch
                self.engine.run_steps(n, host_work=self._shuffle_ahead)
            else:
                self.engine.run_steps(n)
            self.left -= n
            k -= n
