#!/usr/bin/env python3
"""Timings of the per-step exchange forms with N in-process ranks on ONE GPU (no time-slicing):
parallel/inproc.py.  Prints one JSON object:

    python tools/inproc_pair.py [--ranks 2] [--steps 20] [--warmup 5] [--reps 5] [--long 200]

For each form - local (no exchange), xgmi-pull / xgmi-rsag (the serial one-launch exchange),
xgmi-pull-pers / xgmi-rsag-pers (the exchange inside the persistent launch) - it reports the
median over ``reps`` windows of the wall and event-timed us/step of a driver-shaped window
(``--steps`` / ``--warmup``, one exact-size graph replay per rank, as bench.py times it) and of a
``--long`` window, plus the per-step exchange wait measured inside the kernels (median / p99 /
max, max over ranks), and a one-engine local baseline ("single").  ``pers_overhead_us`` = the
-pers form's us/step minus the concurrent local persistent step's (<= 3 us,
or the -pers forms leave the A/B's ORDER).  Every form must finish with no failed wait and with
parameters bit-identical to the serial pull exchange's (checked here too: ``bitwise``).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.data.datasets import SYNTH_NOISE_HARD  # noqa: E402
from distributed_neural_network_amd.models.network import init_arena  # noqa: E402
from distributed_neural_network_amd.parallel import inproc  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402

FORMS = ("local", "xgmi-pull", "xgmi-rsag", "xgmi-pull-pers", "xgmi-rsag-pers")


def trace(engines, groups, runner, form: str, steps: int = 64, reps: int = 5) -> dict:
    """Diagnostic (--trace): where the exchange forms spend their time.  Per-block exchange waits
    (the wait ring: per step, the longest wave wait of each grad_reduce block; medians over the
    steps of block categories) and sample block 0's per-step start times on every rank (stamps,
    s_memrealtime 100 MHz), over ``reps`` launches of ``steps`` steps."""
    dev = engines[0].device
    inproc.set_form(engines, groups, form)
    bufs = [torch.zeros(4096 + 64, dtype=torch.int64, device=dev) for _ in engines]
    for e, b in zip(engines, bufs):
        e._pipe_stamps = b.data_ptr()
    runner.begin()
    runner.prepare(steps)
    cats = {"mlp_tiles": range(0, 64), "mlp_bias": range(64, 68), "conv1": range(68, 76), "conv2": range(76, 113)}
    out = {"form": form, "cats": {}, "step_starts": [], "skew_us": []}
    per_cat = {k: [] for k in cats}
    for _ in range(reps):
        if runner.left < steps:
            runner.begin()
        for g in groups:
            g.reset_wait_stats()
        for b in bufs:
            b.zero_()
        runner.run(steps)
        torch.cuda.synchronize(dev)
        ring, nblk, waves = engines[0].ext.xgmi_wait_ring()
        for g in groups:
            if g.wait is None:
                continue
            w = g.wait.view(ring, nblk, waves).cpu()
            st = (w >> 32) & 0xffffffff
            tk = (w & 0xffffffff).double() / 100.0
            newest = int(st.max())
            for k, blks in cats.items():
                for s_ in range(newest - steps + 2, newest + 1):  # (the launch's steps; the first skipped)
                    m = st[s_ % ring, list(blks)] == s_
                    if bool(m.any()):
                        per_cat[k].append(float(torch.where(m, tk[s_ % ring, list(blks)], torch.zeros(())).max()))
        starts = [b.cpu().numpy()[2048:2048 + steps].astype(np.float64) for b in bufs]
        t0 = min(x[0] for x in starts)
        out["step_starts"].append([[round((v - t0) * 0.01, 2) for v in x[:12]] for x in starts])
        out["skew_us"].append([round(float(np.median(np.abs(starts[0] - x))) * 0.01, 2) for x in starts[1:]])
        out["period_us"] = [round(float(np.median(np.diff(x))) * 0.01, 2) for x in starts]
    for k, v in per_cat.items():
        if v:
            out["cats"][k] = {"median": round(float(np.median(v)), 2), "p90": round(float(np.quantile(v, 0.9)), 2)}
    for e in engines:
        e._pipe_stamps = 0
        e.invalidate_graphs()
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--long", type=int, default=200)
    ap.add_argument("--spin", type=int, default=200)
    ap.add_argument("--forms", default=",".join(FORMS))
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp32"))
    ap.add_argument("--trace", default="", help="diagnostic: per-block waits + per-step starts of these forms")
    a = ap.parse_args()
    n = a.ranks
    train = synthetic(50_000, 0, True, noise=SYNTH_NOISE_HARD)
    shard = len(train) // n
    rng = np.random.default_rng(0)
    orders = [(r * shard + rng.permutation(shard)).astype(np.int32) for r in range(n)]
    arena = init_arena(seed=0)
    engines = [HipEngine(batch=a.batch, arena=arena, graph_chunk=64, dtype=a.dtype) for _ in range(n)]
    for e in engines:
        e.attach(train)
    groups = inproc.build_pair(engines, record_waits=True)
    runner = inproc.PairRunner(engines, orders)
    out = {"ranks": n, "dtype": a.dtype, "batch": a.batch, "steps": a.steps, "warmup": a.warmup, "reps": a.reps, "long": a.long,
           "device": torch.cuda.get_device_name(0), "forms": {}}

    def timed(steps: int, warm: int) -> tuple[float, float]:
        walls, gpus = [], []
        for _ in range(a.reps):
            if runner.left < warm + steps:
                runner.begin()
            runner.run(warm)
            w, g = runner.window(steps)
            walls.append(w)
            gpus.append(g)
        return statistics.median(walls), statistics.median(gpus)

    if a.trace:
        res = [trace(engines, groups, runner, f) for f in a.trace.split(",")]
        inproc.close(engines, groups)
        runner.release()
        print(json.dumps({"trace": res}))
        return
    p0 = [(e.master.clone(), e.mom.clone()) for e in engines]
    finals = {}
    for form in a.forms.split(","):
        inproc.set_form(engines, groups, form)
        for e, (m, mo) in zip(engines, p0):
            with torch.no_grad():
                e.master.copy_(m)
                e.mom.copy_(mo)
            e.params_changed()
            e.epoch_stats(reset=True)
            e.pipe_err.zero_()
        for g in groups:
            g.clear_error()
        # bit-identity run: the same 2 x 17 steps from the same start on every form (graphs captured
        # first: a capture synchronizes the device, which a peer's replay waiting on this rank's
        # granules would turn into a timed-out wait)
        runner.begin()
        runner.prepare(17)
        runner.run(17)
        runner.begin()
        runner.run(17)
        torch.cuda.synchronize()
        finals[form] = [(e.master.cpu(), e.mom.cpu()) for e in engines]
        # timings (each window inside one epoch, exact-size graph, warmup right before it)
        runner.begin()
        runner.prepare(a.steps)
        runner.run(a.spin)
        for g in groups:
            g.reset_wait_stats()
        w20, g20 = timed(a.steps, a.warmup)
        waits = [g.wait_stats() for g in groups] if form != "local" else [None]
        runner.begin()
        runner.prepare(a.long)
        wl, gl = timed(a.long, max(a.warmup, 20))
        torch.cuda.synchronize()
        failed = any(e.pipe_failed() for e in engines) or (form != "local" and any(g.failed() for g in groups))
        pers = all(e._pers_ok() for e in engines)
        wt = None
        if waits and waits[0] is not None:
            wt = {k: round(max(w[k] for w in waits if w), 3) for k in ("median", "p99", "max")}
        out["forms"][form] = {"window_us": round(w20, 3), "window_gpu_us": round(g20, 3), "long_us": round(wl, 3),
                              "long_gpu_us": round(gl, 3), "persistent_launch": pers, "wait_failed": failed,
                              "exchange_wait_us": wt}
        print(f"[inproc] {form}: window {w20:.2f} us/step (gpu {g20:.2f}), long {wl:.2f} (gpu {gl:.2f}), "
              f"persistent {pers}, waits {wt}, failed {failed}", file=sys.stderr, flush=True)
    ref = finals.get("xgmi-pull")
    if ref is not None:
        out["bitwise"] = {f: all(torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]) for x, y in zip(ref, v))
                          for f, v in finals.items() if f != "local"}
        out["replicas_identical"] = {f: all(torch.equal(v[0][0], x[0]) for x in v[1:]) for f, v in finals.items()
                                     if f != "local"}
    loc = out["forms"].get("local")
    if loc:
        out["pers_overhead_us"] = {f: round(v["window_us"] - loc["window_us"], 3) for f, v in out["forms"].items()
                                   if f.endswith("-pers")}
        out["pers_overhead_long_us"] = {f: round(v["long_us"] - loc["long_us"], 3) for f, v in out["forms"].items()
                                        if f.endswith("-pers")}
    inproc.close(engines, groups)
    runner.release()
    # one engine alone (the 1-GPU bench's step), for scale
    e1 = HipEngine(batch=a.batch, arena=arena, graph_chunk=64, dtype=a.dtype)
    e1.attach(train)
    r1 = inproc.PairRunner([e1], [orders[0]])
    runner = r1
    r1.begin()
    r1.prepare(a.steps)
    r1.run(a.spin)
    w20, g20 = timed(a.steps, a.warmup)
    out["single"] = {"window_us": round(w20, 3), "window_gpu_us": round(g20, 3)}
    r1.release()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
