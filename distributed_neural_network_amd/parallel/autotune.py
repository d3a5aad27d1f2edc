"""Start-up A/B of the per-step gradient all-reduce (multi-GPU bench, trainer ``--allreduce auto``).

Why measure instead of guess: at 62,006 parameters the per-step collective is a few
microseconds of xGMI wire time next to a ~20 us step, so which transport wins is decided by
latency terms that depend on the node (link count, RCCL's protocol choice, how far apart the
ranks' steps start) - SURVEY.md §5.8 "measure ... and pick per message size".  The reference
timed its own communication (data_parallelism_train.py:116-120, 209-213, 228-231); this
measures the candidates on the real node, in the real captured step, before the timed run:

* every candidate path (``StepAllReduce.PATHS``) is installed collectively - its own self-test
  included - on the same start parameters, graphs captured, ``warmup`` steps run, then
  ``steps`` steps timed between barrier + device sync; the per-rank time's MAX over ranks is
  the candidate's cost, and a candidate counts only if it installed and finished without a
  failed wait on EVERY rank;
* ``local`` (no all-reduce at all) is timed the same way as the baseline that the
  communication overhead of each path is read against; it is never selectable;
* two rounds in alternating order (the min per path), so clock ramp-up does not favour the
  path that happens to run last;
* every rank adopts the same winner (the decision is made from all-reduced numbers only), the
  parameters and momentum are restored, and the losing paths leave nothing installed.
"""
from __future__ import annotations

import math
import time
from typing import Callable

import torch

ORDER = ("xgmi-pull", "xgmi-rsag", "rccl", "rccl-overlap", "xgmi-pull-ovl", "xgmi-rsag-ovl")
# opt-in (--grad-comm bf16): the xGMI exchanges with bf16 gradient granules - half the link
# bytes, lower-precision gradients, so never a candidate unless asked for
BF16_PATHS = ("xgmi-pull-bf16", "xgmi-rsag-bf16")
RANK = ORDER + BF16_PATHS  # tie-break order


def choose(results: dict[str, dict]) -> str | None:
    """The winner among selectable paths: lowest max-over-ranks us/step among those that passed
    on every rank; ties go to the earlier entry of ``ORDER``.  ``local`` never wins."""
    ok = {k: v["us_per_step"] for k, v in results.items()
          if k != "local" and v.get("ok") and v.get("us_per_step") is not None and math.isfinite(v["us_per_step"])}
    if not ok:
        return None
    return min(ok, key=lambda k: (ok[k], RANK.index(k) if k in RANK else len(RANK)))


def _sync(engine) -> None:
    if engine.device.type == "cuda":
        torch.cuda.synchronize(engine.device)


def _measure(comm, engine, run: Callable[[int], None], steps: int, warmup: int) -> tuple[float, bool]:
    """(max-over-ranks us/step, passed on every rank) of the installed path."""
    if hasattr(engine, "prepare_graphs"):
        engine.prepare_graphs()
    run(warmup)
    comm.barrier()
    _sync(engine)
    t0 = time.perf_counter()
    run(steps)
    _sync(engine)
    comm.barrier()
    _sync(engine)
    dt = time.perf_counter() - t0
    failed = getattr(engine.grad_sync, "failed", None)
    bad = bool(failed()) if failed is not None else False
    ok = all(v == 0.0 for v in comm.gather_scalars(1.0 if bad else 0.0))
    return 1e6 * comm.reduce_scalar(dt, "max") / steps, ok


def allreduce_ab(policy, engine, run: Callable[[int], None], steps: int = 300, warmup: int = 40,
                 rounds: int = 2, candidates: tuple[str, ...] = ORDER) -> dict:
    """Collective (every rank calls it with the same arguments).  Times every candidate,
    installs the winner on ``engine`` (``policy.path`` pins it for later re-attaches) and
    returns {"allreduce_ab": {path: us_per_step | None}, "allreduce": winner,
    "local_us_per_step": ..., "failed": [...]}."""
    comm = policy.comm
    snap = (engine.master.detach().clone(), engine.mom.detach().clone())

    def restore() -> None:
        with torch.no_grad():
            engine.master.copy_(snap[0])
            engine.mom.copy_(snap[1])
        engine.params_changed()
        engine.epoch_stats(reset=True)

    results: dict[str, dict] = {}
    names = ("local",) + tuple(candidates)
    for rnd in range(rounds):
        seq = names if rnd % 2 == 0 else tuple(reversed(names))
        for name in seq:
            if results.get(name, {}).get("ok") is False:
                continue  # failed once: not tried again
            ok = policy.install(engine, name)
            if not ok:
                results[name] = {"ok": False, "us_per_step": None, "why": "install / self-test failed"}
                continue
            restore()
            us, passed = _measure(comm, engine, run, steps, warmup)
            if not passed:
                # a wait timed out somewhere: the sticky error words stay set and the group's
                # step counters may be out of step - drop the group (rebuilt if chosen later)
                policy._drop_xgmi_group()
                results[name] = {"ok": False, "us_per_step": None, "why": "a wait failed during the timed steps"}
                continue
            prev = results.get(name, {}).get("us_per_step")
            results[name] = {"ok": True, "us_per_step": us if prev is None else min(prev, us)}
    win = choose(results)
    engine.grad_sync = None
    if win is None or not policy.install(engine, win):
        win = None
        policy.path = None
        policy.attach(engine)  # the default path (and its fallbacks)
    else:
        policy.path = win
    restore()
    return {"allreduce_ab": {k: (round(v["us_per_step"], 3) if v.get("us_per_step") is not None else None)
                             for k, v in results.items() if k != "local"},
            "local_us_per_step": (round(results["local"]["us_per_step"], 3)
                                  if results.get("local", {}).get("us_per_step") is not None else None),
            "allreduce": policy.installed(engine),
            "failed": sorted(k for k, v in results.items() if not v.get("ok"))}


__all__ = ["BF16_PATHS", "ORDER", "allreduce_ab", "choose"]
