"""Trainer-level handling of a timed-out in-launch step wait, on the CPU:
the engine reports the timeout at the epoch end (StepWaitTimeout), the trainer restores the
epoch's snapshot, steps the engine down (``degrade``) and redoes the epoch - the run finishes with
the parameters of a run that never timed out.  (The GPU form, with a forced device-side timeout,
is tests/test_degrade_gpu.py.)"""
import numpy as np
import torch

from distributed_neural_network_amd.runtime import CpuEngine
from distributed_neural_network_amd.train import parse, trainer

ARGS = ["--epochs", "3", "--batch-size", "32", "--train-samples", "512", "--test-samples", "64", "--device", "cpu",
        "--lr", "0.01", "--seed", "4"]


class _FlakyEngine(CpuEngine):
    """A CPU engine whose first epoch-1 run 'times out' in-launch: it even corrupts its parameters,
    as a real timed-out launch may, so only a restore + redo gives the right result."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.levels = ["persistent"]
        self.epochs_begun = 0
        self.failed = False

    def begin_epoch(self, order):
        self.epochs_begun += 1
        super().begin_epoch(order)

    def run_steps(self, n):
        super().run_steps(n)
        if self.epochs_begun == 2 and self.levels == ["persistent"]:
            self.failed = True
            with torch.no_grad():
                self.master.add_(1.0)

    def step_wait_failed(self):
        return self.failed

    def degrade(self):
        self.failed = False
        self.levels.append("pipelined")
        return "pipelined"


def _run(monkeypatch, engine_cls, args):
    made = []

    def fake_make_engine(device, batch, lr, momentum, arena=None, seed=None, **kw):
        from distributed_neural_network_amd.models.network import init_arena
        e = engine_cls(batch, lr, momentum, arena=init_arena(seed))
        made.append(e)
        return e

    monkeypatch.setattr(trainer, "make_engine", fake_make_engine)
    cfg = parse("data-parallel", args)
    out = trainer.Trainer(cfg).run()
    return made[0], out


def test_step_wait_timeout_restores_degrades_and_redoes_the_epoch(monkeypatch, capsys, tmp_path):
    monkeypatch.chdir(tmp_path)
    flaky, out = _run(monkeypatch, _FlakyEngine, ARGS)
    log = capsys.readouterr().out
    assert "stepping down to the pipelined step and redoing epoch 1" in log, log
    assert flaky.levels == ["persistent", "pipelined"] and flaky.epochs_begun == 4
    assert [h["epoch"] for h in out["history"]] == [0, 1, 2]
    ref, _ = _run(monkeypatch, CpuEngine, ARGS)
    assert torch.equal(flaky.master, ref.master) and torch.equal(flaky.mom, ref.mom)
