"""Step runner that crosses epoch boundaries (bench windows, the all-reduce A/B)."""
from __future__ import annotations


class EpochCursor:
    """Feeds k optimizer steps to the engine, starting a new shuffled epoch (policy epoch_end /
    epoch_start + ``engine.begin_epoch``) whenever one ends - no step is skipped."""

    def __init__(self, engine, sampler, policy, batch: int) -> None:
        self.engine, self.sampler, self.policy, self.batch = engine, sampler, policy, batch
        self.epoch = -1
        self.left = 0
        self.steps_per_epoch = sampler.steps(batch)

    def _next_epoch(self) -> None:
        if self.epoch >= 0:
            self.policy.epoch_end(self.engine, self.epoch)
        self.epoch += 1
        self.policy.epoch_start(self.engine, self.epoch)
        self.engine.begin_epoch(self.sampler.order(self.epoch))
        self.left = self.steps_per_epoch

    def run(self, k: int) -> None:
        while k > 0:
            if self.left == 0:
                self._next_epoch()
            n = min(k, self.left)
            self.engine.run_steps(n)
            self.left -= n
            k -= n
