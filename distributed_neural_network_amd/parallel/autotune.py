"""Start-up A/B of the per-step gradient all-reduce (multi-GPU bench, trainer ``--allreduce ab``).

Why measure instead of guess: at 62,006 parameters the per-step collective is a few
microseconds of xGMI wire time next to a ~20 us step, so which transport wins is decided by
latency terms that depend on the node (link count, RCCL's protocol choice, how far apart the
ranks' steps start) - SURVEY.md §5.8 "measure ... and pick per message size".  The reference
timed its own communication (data_parallelism_train.py:116-120, 209-213, 228-231); this
measures the candidates on the real node, in the real captured step, before the timed run:

* every candidate path (``StepAllReduce.PATHS``) is installed collectively - its own self-test
  included - on the same start parameters;
* after ``spin`` untimed steps (the GPU's clocks ramp up, as they have before bench.py's window),
  it is timed with EXACTLY the shape of bench.py's timed window: inside one epoch (a fresh one
  when the rest of the current epoch cannot hold the window), the window's step count as ONE
  exact-size graph replay, ``warmup`` steps right before it, bracketed by barrier + device
  sync on both sides; ``reps`` windows per round, the median per-rank time, MAX over ranks.
  (Round 3 timed 300 steps as power-of-two chunk replays across epoch boundaries and read
  3.5-4x the timed window's cost for the same path);
* ``local`` (no all-reduce at all) is timed the same way as the baseline that the
  communication overhead of each path is read against; it is never selectable;
* two rounds in alternating order (the min per path), so clock ramp-up does not favour the
  path that happens to run last;
* FAULT-CONTAINED: a candidate whose install, self-test or timing raises on any rank (an RCCL
  init error or timeout, a failed xGMI wait) is voted failed on every rank and lands in
  ``failed`` with its reason; the epoch-boundary error vote is deferred for the whole A/B
  (``lazy_check``) so it cannot escape mid-candidate.  Only "no path at all" is fatal;
* every rank adopts the same winner (the decision is made from all-reduced numbers only), the
  parameters and momentum are restored, and the losing paths leave nothing installed.
"""
from __future__ import annotations

import inspect
import math
import os
import statistics
import sys
import time
from typing import Callable, Optional

import torch

# The default candidates.  The exchange inside the persistent launch ("-pers") left this list in
# round 6 (kept only if it costs <= 3 us/step over the local persistent step):
# with two ranks resident side by side on one GPU and no time-slicing (tools/inproc_pair.py,
# profiles/r6/inproc/) it costs 67 us/step over that step in the 20/5 window (84.6 vs 17.8) and
# loses to the serial one-launch exchange (52.1) in every window length.  DNN_AB_PERS=1 adds it.
ORDER = ("xgmi-pull", "xgmi-rsag", "rccl", "rccl-overlap")
PERS_PATHS = ("xgmi-pull-pers", "xgmi-rsag-pers")
# opt-in (--grad-comm bf16): the xGMI exchanges with bf16 gradient granules - half the link
# bytes, lower-precision gradients, so never a candidate unless asked for
BF16_PATHS = ("xgmi-pull-bf16", "xgmi-rsag-bf16")
RANK = PERS_PATHS + ORDER + BF16_PATHS  # tie-break order (a -pers form first: no kernel boundary)


def default_candidates(grad_comm: str = "fp32") -> tuple[str, ...]:
    """The A/B's candidate list: ORDER, + PERS_PATHS first with DNN_AB_PERS=1, + BF16_PATHS when
    bf16 gradient communication was asked for.  (The in-launch "-ovl" forms lost 3x in every rehearsal and were removed in round 6,
    profiles/r4/ab_rehearsal.)"""
    c = ORDER
    if os.environ.get("DNN_AB_PERS") == "1":
        c = PERS_PATHS + c
    if grad_comm == "bf16":
        c = c + BF16_PATHS
    return c


AB_MAX_STEPS = 256  # bench.py: --ab-steps 0 = the timed window's steps, capped here


def ab_window(steps_per_epoch: int, steps: int | None = None, warmup: int | None = None) -> tuple[int, int]:
    """(timed steps, warmup steps) of one A/B window - ONE rule for bench.py and the trainer (VERDICT
    r5 weak #9: the trainer used fixed 64 / 16 and could pick a different path than the bench):
    the run's own window where it has one (bench.py: --steps / --warmup), capped at AB_MAX_STEPS;
    a trainer, whose window is the epoch, takes as much of an epoch as fits (warmup + steps
    inside one epoch), with a warmup of an eighth of it (at least 1, at most 64)."""
    if steps is not None:
        return max(1, min(int(steps), AB_MAX_STEPS)), max(0, int(warmup or 0))
    spe = max(2, int(steps_per_epoch))
    w = max(1, min(64, spe // 8))
    return max(1, min(AB_MAX_STEPS, spe - w)), w


def budget_default() -> float:
    """Wall budget of the whole A/B (DNN_AB_BUDGET_S, default 240 s): candidates not started
    within it are skipped (and reported failed with that reason), and a candidate's RCCL init
    timeout never exceeds what is left of it."""
    return float(os.environ.get("DNN_AB_BUDGET_S", "240"))


def rccl_margin() -> float:
    """Relative margin within which RCCL is preferred to a faster xGMI path (``DNN_AB_RCCL_MARGIN``,
    default 0.03): SURVEY.md §5.8 makes the custom IPC exchange a fallback for when RCCL's
    small-message latency IS the bottleneck, so a win inside the A/B's noise does not count as
    one."""
    return float(os.environ.get("DNN_AB_RCCL_MARGIN", "0.03"))


def choose(results: dict[str, dict], margin: float | None = None) -> str | None:
    """The winner among selectable paths: lowest max-over-ranks us/step among those that passed
    on every rank; ties go to the earlier entry of ``ORDER``.  ``local`` never wins.  An RCCL path
    within ``margin`` (relative, ``rccl_margin()``) of the fastest path is preferred to it."""
    ok = {k: v["us_per_step"] for k, v in results.items()
          if k != "local" and v.get("ok") and v.get("us_per_step") is not None and math.isfinite(v["us_per_step"])}
    if not ok:
        return None
    best = min(ok, key=lambda k: (ok[k], RANK.index(k) if k in RANK else len(RANK)))
    margin = rccl_margin() if margin is None else margin
    rc = [k for k in ok if k.startswith("rccl")]
    if rc and not best.startswith("rccl"):
        r = min(rc, key=lambda k: (ok[k], RANK.index(k)))
        if ok[r] <= ok[best] * (1.0 + margin):
            return r
    return best


def _sync(engine) -> None:
    if engine.device.type == "cuda":
        torch.cuda.synchronize(engine.device)


def window(comm, engine, cur, steps: int) -> float:
    """One timed window exactly as bench.py times it: barrier + device sync, ``steps`` steps,
    device sync + barrier + device sync (one rank: the device sync).  Returns this rank's seconds."""
    comm.barrier()
    _sync(engine)
    t0 = time.perf_counter()
    cur.run(steps)
    _sync(engine)
    if comm.distributed:
        comm.barrier()
        _sync(engine)
    return time.perf_counter() - t0


def prepare_window(engine, cur, steps: int, warmup: int) -> None:
    """Put the cursor where a ``warmup + steps`` window fits inside one epoch (a fresh epoch if
    the rest of this one is too short) and capture the chunk graphs + the exact-size graph of
    the window (bench.py:153-157).  Capture happens here, outside any timed region."""
    if cur.left < warmup + steps and cur.steps_per_epoch >= warmup + steps:
        cur.left = 0
        cur._next_epoch()
    elif cur.left == 0:
        cur._next_epoch()
    if hasattr(engine, "prepare_graphs"):
        fits = steps <= min(512, cur.left - warmup)
        if "exact" in inspect.signature(engine.prepare_graphs).parameters:
            engine.prepare_graphs(exact=(steps,) if fits else ())
        else:  # engines without exact-size graphs (layer engine)
            engine.prepare_graphs()


def _measure(comm, engine, cur, steps: int, warmup: int, reps: int, spin: int) -> tuple[float, bool]:
    """(max-over-ranks us/step, passed on every rank) of the installed path.  ``spin`` steps run
    first, untimed: a candidate installed on an idle GPU would otherwise be timed at low clocks
    (bench.py's window follows the full-test-set evaluation, a clocked-up GPU; the 2-rank
    rehearsal timed the same path 3.4x slower in the A/B than in the window without this)."""
    prepare_window(engine, cur, steps, warmup)
    cur.run(spin)
    times = []
    for _ in range(reps):
        prepare_window(engine, cur, steps, warmup)
        cur.run(warmup)
        times.append(window(comm, engine, cur, steps))
    if os.environ.get("DNN_AB_DEBUG") == "1":
        print(f"[ab] rank {comm.rank}: windows {[round(1e6 * t / steps, 2) for t in times]} us/step", file=sys.stderr,
              flush=True)
    dt = statistics.median(times)
    failed = getattr(engine.grad_sync, "failed", None)
    bad = bool(failed()) if failed is not None else False
    ok = all(v == 0.0 for v in comm.gather_scalars(1.0 if bad else 0.0))
    return 1e6 * comm.reduce_scalar(dt, "max") / steps, ok


def _agree(comm, ok: bool) -> bool:
    return all(v == 1.0 for v in comm.gather_scalars(1.0 if ok else 0.0))


def allreduce_ab(policy, engine, cur, steps: int = 20, warmup: int = 5, rounds: int = 2, reps: int = 3,
                 candidates: tuple[str, ...] = ORDER, log: Optional[Callable[[str], None]] = None,
                 rccl_init_timeout_s: float = 60.0, spin: int = 200, budget_s: float | None = None,
                 rccl_init_after_xgmi_s: float = 15.0) -> dict:
    """Collective (every rank calls it with the same arguments).  ``cur`` is the run's
    ``EpochCursor``.  Times every candidate, installs the winner on ``engine`` (``policy.path``
    pins it for later re-attaches) and returns {"allreduce_ab": {path: us_per_step | None},
    "allreduce": winner, "local_us_per_step": ..., "failed": [...], "why": {path: reason},
    "ab_wall_s": seconds, "variant": {path: step form it was timed with}}.

    Bounded: the whole A/B has a wall budget (``budget_s``, default
    ``budget_default()``); a candidate is started only while the budget lasts (decided from the
    max elapsed time over ranks, so every rank skips the same ones), a candidate whose install +
    timing ran past it is marked failed, and the RCCL init timeout of a candidate is capped by
    the budget left - and by ``rccl_init_after_xgmi_s`` once an xGMI path has passed (RCCL can
    then only win by being fast, and a slow init says it will not)."""
    comm = policy.comm
    budget = budget_default() if budget_s is None else float(budget_s)
    t_start = time.perf_counter()
    say = log or (lambda s: None)
    snap = (engine.master.detach().clone(), engine.mom.detach().clone())

    def restore() -> None:
        with torch.no_grad():
            engine.master.copy_(snap[0])
            engine.mom.copy_(snap[1])
        engine.params_changed()
        engine.epoch_stats(reset=True)

    results: dict[str, dict] = {}
    names = ("local",) + tuple(candidates)
    lazy = getattr(policy, "lazy_check", False)
    policy.lazy_check = True  # an xGMI wait failure is voted per candidate below, not at an epoch end
    tmo = os.environ.get("DNN_RCCL_INIT_TIMEOUT_S")
    variant: dict[str, str] = {}
    try:
        for rnd in range(rounds):
            seq = names if rnd % 2 == 0 else tuple(reversed(names))
            for name in seq:
                if results.get(name, {}).get("ok") is False:
                    continue  # failed once: not tried again
                left = budget - comm.reduce_scalar(time.perf_counter() - t_start, "max")
                if left <= 0:
                    if name not in results:
                        results[name] = {"ok": False, "us_per_step": None, "why": f"skipped: A/B wall budget "
                                                                                   f"({budget:.0f} s) spent"}
                        say(f"A/B {name}: skipped (budget spent)")
                    continue
                xgmi_ok = any(v.get("ok") for k, v in results.items() if k.startswith("xgmi"))
                cap = min(float(tmo or 1e9), rccl_init_timeout_s, max(1.0, left))
                if xgmi_ok:
                    cap = min(cap, rccl_init_after_xgmi_s)
                os.environ["DNN_RCCL_INIT_TIMEOUT_S"] = str(cap)
                policy.ab_deadline = time.time() + left  # (candidates may bound their own set-up by it)
                t0 = time.perf_counter()
                why = ""
                try:
                    ok = bool(policy.install(engine, name))
                    if not ok:
                        why = getattr(policy, "install_why", "") or "install / self-test failed"
                except Exception as e:  # contained: this candidate fails, the A/B goes on
                    ok, why = False, f"install raised {type(e).__name__}: {e}"
                if not _agree(comm, ok):
                    why = why or "failed on another rank"
                    results[name] = {"ok": False, "us_per_step": None, "why": why}
                    _drop(policy, engine, name)
                    say(f"A/B {name}: FAILED ({why}) after {time.perf_counter() - t0:.2f}s")
                    continue
                restore()
                passed, us = True, None
                try:
                    us, passed = _measure(comm, engine, cur, steps, warmup, reps, spin)
                    if not passed:
                        why = "a wait failed during the timed steps"
                except Exception as e:
                    passed, why = False, f"timing raised {type(e).__name__}: {e}"
                if not _agree(comm, passed):
                    results[name] = {"ok": False, "us_per_step": None, "why": why or "failed on another rank"}
                    # sticky error words stay set and the group's step counters may be out of
                    # step: drop the group (rebuilt if another xGMI path is tried later)
                    _drop(policy, engine, name)
                    say(f"A/B {name}: FAILED ({results[name]['why']})")
                    continue
                spent = comm.reduce_scalar(time.perf_counter() - t0, "max")
                if spent > left:  # ran past the whole A/B's budget: not selectable
                    results[name] = {"ok": False, "us_per_step": None,
                                     "why": f"over the A/B wall budget ({spent:.1f} s for this candidate, "
                                            f"{left:.1f} s left)"}
                    _drop(policy, engine, name)
                    say(f"A/B {name}: FAILED ({results[name]['why']})")
                    continue
                variant[name] = step_variant(engine)
                prev = results.get(name, {}).get("us_per_step")
                results[name] = {"ok": True, "us_per_step": us if prev is None else min(prev, us)}
                say(f"A/B {name}: {us:.3f} us/step (round {rnd}, {time.perf_counter() - t0:.2f}s incl. install)")
        win = choose(results)
        engine.grad_sync = None
        installed = False
        if win is not None:
            try:
                installed = bool(policy.install(engine, win))
            except Exception as e:
                say(f"A/B winner {win} could not be re-installed: {type(e).__name__}: {e}")
            installed = _agree(comm, installed)
        if not installed:
            win = None
            policy.path = None
            policy.attach(engine)  # the default path (and its fallback chain)
        else:
            policy.path = win
        restore()
    finally:
        policy.lazy_check = lazy
        policy.ab_deadline = None
        if tmo is None:
            os.environ.pop("DNN_RCCL_INIT_TIMEOUT_S", None)
        else:
            os.environ["DNN_RCCL_INIT_TIMEOUT_S"] = tmo
    return {"allreduce_ab": {k: (round(v["us_per_step"], 3) if v.get("us_per_step") is not None else None)
                             for k, v in results.items() if k != "local"},
            "local_us_per_step": (round(results["local"]["us_per_step"], 3)
                                  if results.get("local", {}).get("us_per_step") is not None else None),
            "allreduce": policy.installed(engine),
            "failed": sorted(k for k, v in results.items() if not v.get("ok")),
            "why": {k: v["why"] for k, v in results.items() if not v.get("ok")},
            "ab_wall_s": round(comm.reduce_scalar(time.perf_counter() - t_start, "max"), 3),
            "variant": variant}


def step_variant(engine) -> str:
    """The step form a candidate was timed with (the no-all-reduce baseline may run
    the persistent step while a candidate runs the serial one): persistent / pipelined / serial."""
    if getattr(engine, "_pers_ok", lambda: False)():
        return "persistent"
    if getattr(engine, "_pipe_ok", lambda: False)():
        return "pipelined"
    return "serial"


def _drop(policy, engine, name: str) -> None:
    """Leave nothing of a failed candidate installed."""
    engine.grad_sync = None
    if name.startswith("xgmi") and hasattr(policy, "_drop_xgmi_group"):
        try:
            policy._drop_xgmi_group()
        except Exception as e:
            print(f"[ab] dropping the xGMI group after {name} failed: {e}", file=sys.stderr, flush=True)
    if name.startswith("rccl"):
        nat = getattr(policy.comm, "native", None)
        if nat is not None:
            try:
                nat.abort()
            except Exception:
                pass
            policy.comm.native = None


__all__ = ["AB_MAX_STEPS", "BF16_PATHS", "ORDER", "PERS_PATHS", "ab_window", "allreduce_ab", "budget_default", "choose",
           "default_candidates", "prepare_window", "rccl_margin", "step_variant", "window"]


# -- how the persistent window is launched ----------------------------------------------------
LAUNCH_PATHS = ("direct-aql", "graph")


def launch_margin() -> float:
    """Relative margin within which the direct AQL dispatch is kept against a faster graph replay
    (``DNN_LAUNCH_MARGIN``, default 0.005): its launch + completion path is the shorter one
    (profiles/r6/aql/), so a graph win inside the A/B's noise does not count as one."""
    return float(os.environ.get("DNN_LAUNCH_MARGIN", "0.005"))


def launch_ab(comm, engine, cur, steps: int = 20, warmup: int = 5, rounds: int = 4, reps: int = 3,
              spin: int = 500, log: Optional[Callable[[str], None]] = None) -> dict:
    """Start-up A/B of the persistent window's launch path, the counterpart of ``allreduce_ab`` for
    engines whose window runs without a per-step all-reduce (collective: every rank calls it).
    Times the direct AQL dispatch (csrc/runtime/aql_dispatch.h) and the captured-graph replay with
    the run's own window shape (``_measure``: the bench's bracket, max over ranks), alternating
    over ``rounds``, keeps the faster one on ``engine`` (the direct dispatch within
    ``launch_margin()``) and returns {"launch_ab": {path: median us/step}, "launch": winner,
    "launch_ab_wall_s": seconds}; {} where there is nothing to choose (no AQL queue on this
    device, another engine, the fp32 step or a per-step all-reduce installed).  Like the all-reduce
    A/B, the first candidate runs ``spin`` untimed steps first, so no path is timed at the low
    clocks of a GPU that sat idle through the set-up (a cold 20/5 window is ~0.3 us/step slower:
    profiles/r6/aql/)."""
    say = log or (lambda m: None)
    was = bool(getattr(engine, "direct", False))
    if not was:
        return {}
    if cur is not None:
        prepare_window(engine, cur, steps, warmup)  # (an epoch begun: the step forms are decided)
    if not getattr(engine, "_direct_ok", lambda: False)():
        return {}
    t_start = time.perf_counter()
    res: dict[str, list[float]] = {p: [] for p in LAUNCH_PATHS}
    try:
        for rnd in range(rounds):
            for i, p in enumerate(LAUNCH_PATHS if rnd % 2 == 0 else LAUNCH_PATHS[::-1]):
                engine.direct = p == "direct-aql"
                us, _ = _measure(comm, engine, cur, steps, warmup, reps, spin if rnd == 0 and i == 0 else 0)
                res[p].append(us)
                say(f"launch A/B {p}: {us:.3f} us/step (round {rnd})")
    finally:
        engine.direct = was
    med = {p: round(statistics.median(v), 3) for p, v in res.items()}
    winner = "direct-aql" if med["direct-aql"] <= med["graph"] * (1.0 + launch_margin()) else "graph"
    engine.direct = winner == "direct-aql"
    return {"launch_ab": med, "launch": winner, "launch_ab_wall_s": round(time.perf_counter() - t_start, 3)}
