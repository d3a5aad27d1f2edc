"""Timed-window overhead of a SHORT run (the driver times --steps 20 --warmup 5): the bench's
protocol (W warmup steps, sync, K timed steps, sync) with the K steps issued as
  chunks  - the engine's power-of-two chunk graphs (16 + 4 replays for K = 20)
  exact   - one graph of exactly K steps
  eager   - K x 2 plain launches
repeated R times each (median).  usage: python tools/window_probe.py [K] [W] [R]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_neural_network_amd.data import EpochSampler, synthetic  # noqa: E402
from distributed_neural_network_amd.runtime import HipEngine  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    dev = torch.device("cuda", 0)
    train = synthetic(50_000, 0, True)
    samp = EpochSampler.for_rank(len(train), 0, 1, seed=0, mode="shard")
    eng = HipEngine(batch=64, seed=0, device=dev, graph_chunk=64)
    eng.attach(train)
    eng.begin_epoch(samp.order(0))
    eng.prepare_graphs()
    exact = eng._graph(K) if K & (K - 1) else None  # a non power of two: its own graph
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for mode in ("chunks", "exact", "eager", "chunks"):
        walls, gpus = [], []
        for _ in range(R):
            if eng.steps_per_epoch() - 0 < (W + K) * 2:
                pass
            eng.begin_epoch(samp.order(0))
            eng.run_steps(W)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev0.record()
            if mode == "chunks":
                eng.run_steps(K)
            elif mode == "exact" and exact is not None:
                exact.replay()
            else:
                eng.use_graphs = False
                eng.run_steps(K)
                eng.use_graphs = True
            ev1.record()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            gpus.append(ev0.elapsed_time(ev1) * 1e3)
        res.setdefault(mode, []).append((np.median(walls), np.median(gpus)))
        print(f"{mode:7s} K={K} W={W}: wall {np.median(walls):7.1f} us ({np.median(walls) / K:5.2f}/step)  "
              f"events {np.median(gpus):7.1f} us  min wall {min(walls):7.1f}", flush=True)


if __name__ == "__main__":
    main()
