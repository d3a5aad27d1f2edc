"""Repeat tests/test_engine_gpu.py::test_pipelined_long_run_under_load's comparison many times,
per engine variant, in ONE process: 600 steps next to a side stream of GEMMs, each variant's
master weights against its dtype's serial step, bit for bit.  Prints one line per round and a
per-variant mismatch count (a hand-off race shows up as a rare few-value difference).

    python tools/race_hunt.py [--rounds N] [--variants bf16-pipe,bf16-pers,fp32-pers]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import synthetic  # noqa: E402
from distributed_neural_network_amd.models.network import init_arena  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402

VARIANTS = {"bf16-pipe": (True, False, "bf16"), "bf16-pers": (True, True, "bf16"), "fp32-pers": (False, True, "fp32"),
            "fp32-serial": (False, False, "fp32"), "bf16-serial": (False, False, "bf16")}


CHUNKS = (32, 16, 8, 4)  # run_steps(60)'s own graph decomposition, one call each (--trace)


def run(data, order, pipe, pers, dt, seed_side, load=True, trace=False):
    eng = HipEngine(batch=64, arena=init_arena(seed=6), graph_chunk=32, pipeline=pipe, persist=pers, dtype=dt)
    assert eng.persist == pers
    eng.attach(data)
    side = torch.cuda.Stream()
    g = torch.Generator(device="cuda").manual_seed(seed_side)
    x = torch.randn(2048, 2048, device="cuda", generator=g)
    snaps = []
    for _ in range(10):
        eng.begin_epoch(order)
        with torch.cuda.stream(side):
            for _ in range(4 if load else 0):
                x = torch.tanh(x @ x * 1e-3)
        if trace:
            for k in CHUNKS:
                eng.run_steps(k)
                snaps.append(eng.master.clone())
        else:
            eng.run_steps(60)
    torch.cuda.synchronize()
    assert not eng.pipe_failed()
    return eng.master.cpu(), eng.mom.cpu(), eng.epoch_stats().loss_sum, snaps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--variants", default="bf16-pipe,bf16-pers,fp32-pers")
    ap.add_argument("--no-load", action="store_true", help="no side stream of GEMMs")
    ap.add_argument("--trace", action="store_true", help="snapshot the weights after every chunk: first divergent one")
    args = ap.parse_args()
    data = synthetic(4096, 12)
    order = np.random.default_rng(4).permutation(4096).astype(np.int32)
    ref = {dt: run(data, order, False, False, dt, 0, trace=args.trace) for dt in ("bf16", "fp32")}
    bad = {v: 0 for v in args.variants.split(",")}
    for r in range(args.rounds):
        t0 = time.time()
        for v in bad:
            pipe, pers, dt = VARIANTS[v]
            m, mom, loss, snaps = run(data, order, pipe, pers, dt, r + 1, not args.no_load, args.trace)
            r0 = ref[dt]
            if not (torch.equal(m, r0[0]) and torch.equal(mom, r0[1]) and loss == r0[2]):
                diff = (m != r0[0]).nonzero().flatten()
                bad[v] += 1
                print(f"round {r} {v}: MISMATCH {diff.numel()} master values, first at {diff[:8].tolist()}", flush=True)
                for i, (a, b) in enumerate(zip(snaps, r0[3])):
                    if not torch.equal(a, b):
                        d = (a != b).nonzero().flatten()
                        print(f"   first divergent chunk: epoch {i // len(CHUNKS)}, chunk {CHUNKS[i % len(CHUNKS)]} "
                              f"(steps {sum(CHUNKS[:i % len(CHUNKS)])}..+{CHUNKS[i % len(CHUNKS)]}): {d.numel()} values, "
                              f"first at {d[:8].tolist()}, last at {d[-4:].tolist()}", flush=True)
                        break
        print(f"round {r} done in {time.time() - t0:.1f} s", flush=True)
    print("mismatches per variant:", bad, flush=True)


if __name__ == "__main__":
    main()
