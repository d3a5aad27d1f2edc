#!/usr/bin/env python3
"""Diagnostic: WHEN do the two in-process ranks of the exchange inside the persistent launch part?

    python tools/inproc_diverge.py [--dtype fp32] [--form xgmi-pull-pers] [--reps 3]

For every launch pattern (graph replays of the test's chunks, one-step graphs, eager launches)
and repetition it builds the in-process pair of tests/test_inproc_pair_gpu.py, synchronizes after
every ``run_steps`` call and compares the two ranks' fp32 masters (the exchange makes them
bit-identical by construction).  Prints one JSON object: per run the first call after which the
replicas differ, how many elements, which parameter tensors and a few values (both masters, both
momenta, rank 0's bf16 shadow) - enough to tell a stale operand from a lost update."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.models.network import LAYOUT, init_arena  # noqa: E402
from distributed_neural_network_amd.parallel import inproc  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402


def where(d: torch.Tensor) -> dict:
    return {k: int(((d >= o) & (d < o + LAYOUT.numel(k))).sum()) for k, o in LAYOUT.offsets.items()
            if int(((d >= o) & (d < o + LAYOUT.numel(k))).sum())}


def one(dtype: str, form: str, graphs: bool, chunk: int, pattern: list[int], batch: int, epochs: int) -> dict:
    data = synthetic(2000, 13)
    arena = init_arena(seed=9)
    rng = np.random.default_rng(2)
    engines = [HipEngine(batch=batch, arena=arena, graph_chunk=chunk, use_graphs=graphs, dtype=dtype) for _ in range(2)]
    for e in engines:
        e.attach(data)
    groups = inproc.build_pair(engines, timeout_s=5.0)
    inproc.set_form(engines, groups, form)
    streams = inproc.own_queue_streams(engines)
    out = {"graphs": graphs, "chunk": chunk, "pattern": pattern, "first": None, "calls": 0}
    try:
        call = 0
        for ep in range(epochs):
            orders = [(1000 * r + rng.permutation(1000)).astype(np.int32) for r in range(2)]
            for e, s, o in zip(engines, streams, orders):
                with torch.cuda.stream(s):
                    e.begin_epoch(o)
            if ep == 0:
                for e in engines:
                    e.prepare_graphs()
            for k in pattern:
                for e, s in zip(engines, streams):
                    with torch.cuda.stream(s):
                        e.run_steps(k)
                torch.cuda.synchronize()
                call += 1
                d = (engines[0].master != engines[1].master).nonzero().flatten()
                if d.numel() and out["first"] is None:
                    n = LAYOUT.total
                    i = d[:6]
                    out["first"] = {
                        "epoch": ep, "call": call, "steps_in_call": k, "n": int(d.numel()), "where": where(d.cpu()),
                        "idx": i.tolist(),
                        "master0": engines[0].master[i].tolist(), "master1": engines[1].master[i].tolist(),
                        "mom0": engines[0].mom[i].tolist(), "mom1": engines[1].mom[i].tolist(),
                        "shadow_mismatch": [int((e.shadow[:n] != e.master[:n].to(torch.bfloat16)).sum())
                                            for e in engines],
                        "xp_ctr": [g.xp_ctr[:4].tolist() for g in groups]}
        out["calls"] = call
        out["failed"] = bool(any(e.pipe_failed() for e in engines) or any(g.failed() for g in groups))
        out["final_diff"] = int((engines[0].master != engines[1].master).sum())
    finally:
        inproc.close(engines, groups)
        inproc.release_streams(engines, streams)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--form", default="xgmi-pull-pers")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--runs", default="g8,g1,eager")
    a = ap.parse_args()
    batch = 64 if a.dtype == "bf16" else 32
    spe = -(-1000 // batch)
    runs = {"g8": (True, 8, [5, spe - 5]), "g1": (True, 1, [1] * spe), "eager": (False, 8, [5, spe - 5]),
            "g8split": (True, 8, [1] * spe), "g64": (True, 64, [5, spe - 5])}
    res = []
    for name in a.runs.split(","):
        g, c, p = runs[name]
        for r in range(a.reps):
            o = one(a.dtype, a.form, g, c, p, batch, a.epochs)
            o["run"], o["rep"] = name, r
            print(f"[diverge] {name} rep {r}: first {o['first'] and (o['first']['epoch'], o['first']['call'], o['first']['n'])}"
                  f" final {o['final_diff']} failed {o['failed']}", file=sys.stderr, flush=True)
            res.append(o)
    print(json.dumps({"dtype": a.dtype, "form": a.form, "runs": res}))


if __name__ == "__main__":
    main()
